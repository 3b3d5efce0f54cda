# GPU: the GPU suite on the defaults (lt_giant rows pass, pool counters test),
# then batch 1 / B=64 / ResNet with ORION_MAC_ROWS 0 / 1 (it gates both row fusions)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r05aa.log 2>&1 || { tail -30 gpurun_out/pytest_r05aa.log; exit 1; }
tail -1 gpurun_out/pytest_r05aa.log
PK=none B1=2 BENCH=1 RESNET=1 bash tools/gpu_ab_env.sh r05aa ORION_MAC_ROWS 0 1
