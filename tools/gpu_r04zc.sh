# r04zc: basis-extension target sums in float64 for targets below 2^46
# (BEXT_F64, ORION_BEXT_F64 0/1): GPU suite with it on, then batch 1 and LoLA
# B=64 bench + kernel trace per value
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r04zc.log 2>&1 || { tail -30 gpurun_out/pytest_r04zc.log; exit 1; }
tail -1 gpurun_out/pytest_r04zc.log
for rep in 1 2; do for v in 0 1; do
  ORION_BEXT_F64=$v timeout -k 10 300 python bench.py --batch 1 --steps 50 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/ab_r04zc_b1_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/ab_r04zc_b1_${v}_$rep.log; exit 1; }
  echo "$v batch1 $rep: $(tail -1 gpurun_out/ab_r04zc_b1_${v}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/step")')"
done; done
PARITY=0 NTT=0 BENCH=2 KPROF=1 RESNET=0 bash tools/ab.sh r04zc env ORION_BEXT_F64 0 1
