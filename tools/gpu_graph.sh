# one GPU call: boundary tests (graph capture) + bench with batch-1 / batched graph replay
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02i}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -m gpu --timeout 200 --timeout-method thread tests/test_gpu_boundary.py > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d["batch1"], d["graph_replay"])'
