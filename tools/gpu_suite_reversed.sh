# the GPU suite once in reverse node order (fixtures must not
# depend on test order); usage: bash tools/gpu_suite_reversed.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 120 python -m pytest tests -m gpu --collect-only -q 2>/dev/null | grep "::" | tac > gpurun_out/nodes_rev_$TAG.txt
timeout -k 10 1000 python -u -m pytest -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread $(cat gpurun_out/nodes_rev_$TAG.txt) > gpurun_out/pytest_rev_$TAG.log 2>&1 || { echo "reversed suite failed"; grep -E "FAILED|ERROR" gpurun_out/pytest_rev_$TAG.log | head; tail -40 gpurun_out/pytest_rev_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_rev_$TAG.log
