# GPU: ResNet-20 N=2^16 (configs/resnet.yml) at the given batches, no profiler,
# with the device-pool counters.  usage: bash tools/gpu_resnet.sh TAG [BATCHES="1 4"]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-resnet}
mkdir -p gpurun_out
for b in ${BATCHES:-1 4}; do
  WORKLOAD=resnet20_n16 BATCH=$b timeout -k 10 ${RESNET_TIMEOUT:-400} python -u tools/resnet_bench.py > gpurun_out/${TAG}_resnet_b$b.log 2>&1 || { tail -20 gpurun_out/${TAG}_resnet_b$b.log; exit 1; }
  tail -2 gpurun_out/${TAG}_resnet_b$b.log
done
