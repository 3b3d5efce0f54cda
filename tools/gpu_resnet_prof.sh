# GPU: rocprofv3 kernel trace of one ResNet-20 N=2^16 inference (tools/resnet_bench.py, batch 1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
WORKLOAD=resnet20_n16 BATCH=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn16 -o kt --output-format csv -- python -u tools/resnet_bench.py > gpurun_out/prof_rn16.log 2>&1 || { tail -20 gpurun_out/prof_rn16.log; exit 1; }
tail -2 gpurun_out/prof_rn16.log
