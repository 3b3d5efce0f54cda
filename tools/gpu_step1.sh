set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" 
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 900 python bench.py --steps 3 --warmup 1 > gpurun_out/bench1.log 2>&1; echo "bench rc=$?"
tail -5 gpurun_out/bench1.log
