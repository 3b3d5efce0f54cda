# r04k: INTT -> prologue NTT fusion on the latency kernels (ORION_NTT_IFUSE) and
# the basis-extension target modes (ORION_BEXT_MODES): parity, then A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r04k.log 2>&1 || { tail -30 gpurun_out/pytest_r04k.log; exit 1; }
tail -1 gpurun_out/pytest_r04k.log
for rep in 1 2; do
  for v in 0 1; do
    ORION_NTT_IFUSE=$v timeout -k 10 200 python bench.py --batch 1 --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/r04k_b1_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/r04k_b1_${v}_$rep.log; exit 1; }
    echo "IFUSE=$v batch1 $rep: $(tail -1 gpurun_out/r04k_b1_${v}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/image")')"
  done
done
for v in 0 1; do
  ORION_BEXT_MODES=$v WORKLOAD=resnet20_n16 BATCH=1 timeout -k 10 400 python -u tools/resnet_bench.py > gpurun_out/r04k_resnet_modes$v.log 2>&1 || { tail -20 gpurun_out/r04k_resnet_modes$v.log; exit 1; }
  echo "BEXT_MODES=$v resnet: $(grep workload gpurun_out/r04k_resnet_modes$v.log | tail -1 | cut -c1-160)"
done
