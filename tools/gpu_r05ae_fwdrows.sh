# GPU: the gadget product running the decomposition's forward rows pass too
# (ORION_MAC_FWD_ROWS 0 / 1): the GPU suite with the switch on, then batch 1 /
# B=64 / ResNet-20 N=2^16 alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ORION_MAC_FWD_ROWS=1 timeout -k 10 800 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r05ae_on.log 2>&1 || { tail -30 gpurun_out/pytest_r05ae_on.log; exit 1; }
tail -1 gpurun_out/pytest_r05ae_on.log
PK=none B1=2 BENCH=1 RESNET=1 bash tools/gpu_ab_env.sh r05ae ORION_MAC_FWD_ROWS 0 1
