# one GPU call: parity tests -> bench -> rocprofv3 kernel trace -> PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 900 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
[ "${2:-}" = "noprof" ] && exit 0
bash tools/gpu_prof.sh $TAG
