# r04w: the runtime-switch parity test
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "runtime_switch" --timeout 300 --timeout-method thread > gpurun_out/pytest_r04w.log 2>&1 || { tail -40 gpurun_out/pytest_r04w.log; exit 1; }
tail -8 gpurun_out/pytest_r04w.log
