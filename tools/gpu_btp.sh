set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 500 --timeout-method thread tests/test_gpu_ops.py -k resnet > gpurun_out/pytest_btp2.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_btp2.log; exit 1; }
tail -3 gpurun_out/pytest_btp2.log
LOGN=16 BATCH=1,4 timeout -k 10 300 python -u tools/btp_bench.py > gpurun_out/btp_bench_btp2.log 2>&1 || { echo "btp bench failed"; tail -20 gpurun_out/btp_bench_btp2.log; exit 1; }
LOGN=15 BATCH=1,8 timeout -k 10 300 python -u tools/btp_bench.py >> gpurun_out/btp_bench_btp2.log 2>&1 || { echo "btp bench failed"; tail -20 gpurun_out/btp_bench_btp2.log; exit 1; }
cat gpurun_out/btp_bench_btp2.log
WORKLOAD=resnet20_n16 BATCH=1 timeout -k 10 400 python -u tools/resnet_bench.py > gpurun_out/resnet_n16_btp2.log 2>&1 || { echo "resnet bench failed"; tail -20 gpurun_out/resnet_n16_btp2.log; exit 1; }
cat gpurun_out/resnet_n16_btp2.log
