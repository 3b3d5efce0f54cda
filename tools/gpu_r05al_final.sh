# GPU: round-end check of HEAD -- the GPU suite, smoke(), and the driver's bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05al_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r05al_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r05al_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05al_smoke.log 2>&1 || { tail -20 gpurun_out/r05al_smoke.log; exit 1; }
tail -1 gpurun_out/r05al_smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05al_bench.log 2>&1 || { tail -20 gpurun_out/r05al_bench.log; exit 1; }
tail -1 gpurun_out/r05al_bench.log | cut -c1-300
