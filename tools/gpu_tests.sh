# one GPU call: the GPU test suite (or the given files / -k expression)
# usage: bash tools/gpu_tests.sh TAG [pytest args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r03}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread "${@:-tests}" > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|ERROR" gpurun_out/pytest_$TAG.log | head; tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
