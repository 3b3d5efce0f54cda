# GPU A/B of batch-1 latency (BASELINE configs[2]) and the B=64 line, one gpurun call:
# each variant runs the full bench (extras on: the hipGraph and stream-launched
# batch-1 passes without HIP-event profiling), alternating, REPS times.
#   bash tools/gpu_b1_ab.sh TAG lib V1 V2 ...      library variants (V = product: in-tree library)
#   bash tools/gpu_b1_ab.sh TAG env VAR A B ...    runtime switch VAR=A, VAR=B, ...
# Output: gpurun_out/b1ab_<TAG>_<variant>_<rep>.log and one summary line per run.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:?tag}; MODE=${2:?lib or env}; shift 2
if [ "$MODE" = env ]; then VAR=${1:?variable}; shift; fi
mkdir -p gpurun_out
for r in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    o=gpurun_out/b1ab_${TAG}_${v}_$r.log
    if [ "$MODE" = lib ]; then
      lib=orion_amd/liborion_hip.so; [ "$v" != product ] && lib=orion_amd/_build/liborion_hip_$v.so
      ORION_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $o 2>&1 || { tail -20 $o; exit 1; }
    else
      env "$VAR=$v" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $o 2>&1 || { tail -20 $o; exit 1; }
    fi
    echo "$v $r: $(tail -1 $o | python -c 'import json,sys; d=json.loads(sys.stdin.read()); b=d["batch1"]; print("batch1 graph", b["ms_per_image"], "stream", b["stream_ms_per_image"], "ms; B=64", d["value"], "img/s", d["kernel_ms_per_step"])')"
  done
done
