# GPU: ResNet-20 N=2^16 (configs/resnet.yml) at HEAD, batch 1 and batch 4, no profiler
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in 1 4; do
  WORKLOAD=resnet20_n16 BATCH=$b timeout -k 10 400 python -u tools/resnet_bench.py > gpurun_out/r05am_resnet_b$b.log 2>&1 || { tail -20 gpurun_out/r05am_resnet_b$b.log; exit 1; }
  tail -2 gpurun_out/r05am_resnet_b$b.log
done
