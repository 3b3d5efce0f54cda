# GPU: rocprofv3 kernel-trace stats of the LoLA bench per library variant
# usage: bash tools/gpu_kprof_ab.sh TAG variant...   (product = orion_amd/liborion_hip.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  lib=orion_amd/liborion_hip.so; [ $v != product ] && lib=orion_amd/_build/liborion_hip_$v.so
  ORION_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kp_$TAG -o $v -- python3 bench.py --no-cpu-baseline --no-extras --steps 5 --warmup 2 > gpurun_out/kp_${TAG}_$v.log 2>&1 || { tail -20 gpurun_out/kp_${TAG}_$v.log; exit 1; }
  f=$(find gpurun_out/kp_$TAG -name "${v}_kernel_stats.csv" | head -1)
  python3 - "$f" "$v" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
out = [sys.argv[2], f"total {tot/1e6:.2f} ms"]
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    out.append(f"{r['Name'].split('(')[0].split('::')[-1][:28]} {int(r['Calls'])}x{float(r['AverageNs'])/1e3:.1f}us")
print(" | ".join(out))
PY
done
