# one GPU call: host probe -> GPU tests -> smoke -> bench (1 GPU) -> N-rank rehearsal on the one GPU
# usage: bash tools/gpu_check.sh TAG [pytest -k expression]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02}
KEXPR=${2:-}
mkdir -p gpurun_out
{ nproc; lscpu | grep -E "Model name|Socket|Core|Thread|NUMA node\(s\)"; cat /sys/fs/cgroup/cpu.max 2>/dev/null;
  python -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; free -g | head -2; } > gpurun_out/host_$TAG.txt 2>&1
if [ -n "$KEXPR" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -k "$KEXPR" --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
fi
tail -1 gpurun_out/pytest_$TAG.log
[ "${SKIP_BENCH:-0}" = "1" ] && exit 0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -c 1500 gpurun_out/bench_$TAG.log
ORION_BENCH_REHEARSE=1 timeout -k 10 600 python bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/rehearse2_$TAG.log 2>&1 || { echo "rehearse failed"; tail -20 gpurun_out/rehearse2_$TAG.log; exit 1; }
tail -c 600 gpurun_out/rehearse2_$TAG.log
