set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r03a.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|ERROR" gpurun_out/pytest_r03a.log | head; tail -40 gpurun_out/pytest_r03a.log; exit 1; }
tail -1 gpurun_out/pytest_r03a.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r03a.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_r03a.log; exit 1; }
tail -c 400 gpurun_out/bench_r03a.log
bash tools/sigsegv_probe.sh r03a
