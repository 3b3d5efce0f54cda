# r04q: radix-4 latency NTT passes (NTT2S_R4, product) vs radix-2 (r2 build):
# the whole GPU suite on the product, then batch-1 benches and ResNet-20
# N=2^16 for both builds on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r04q.log 2>&1 || { tail -30 gpurun_out/pytest_r04q.log; exit 1; }
tail -1 gpurun_out/pytest_r04q.log
for rep in 1 2; do
  for v in product r2; do
    lib=orion_amd/liborion_hip.so; [ $v != product ] && lib=orion_amd/_build/liborion_hip_$v.so
    ORION_LIB=$lib timeout -k 10 200 python bench.py --batch 1 --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/r04q_b1_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/r04q_b1_${v}_$rep.log; exit 1; }
    echo "$v batch1 $rep: $(tail -1 gpurun_out/r04q_b1_${v}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/image")')"
  done
done
for v in product r2; do
  lib=orion_amd/liborion_hip.so; [ $v != product ] && lib=orion_amd/_build/liborion_hip_$v.so
  ORION_LIB=$lib WORKLOAD=resnet20_n16 BATCH=1 timeout -k 10 300 python -u tools/resnet_bench.py > gpurun_out/r04q_resnet_$v.log 2>&1 || { tail -20 gpurun_out/r04q_resnet_$v.log; exit 1; }
  echo "$v resnet: $(grep workload gpurun_out/r04q_resnet_$v.log | tail -1 | cut -c90-160)"
done
