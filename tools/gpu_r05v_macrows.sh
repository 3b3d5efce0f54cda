# GPU: keyswitch's gadget product storing the P limbs through the ModDown
# INTT's rows pass (ORION_MAC_ROWS=1, ks_mac_rows_kernel): the GPU suite on
# the defaults, then batch-1 / B=64 / ResNet-20 N=2^16 with the switch 0 / 1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r05v.log 2>&1 || { tail -30 gpurun_out/pytest_r05v.log; exit 1; }
tail -1 gpurun_out/pytest_r05v.log
PK=none B1=2 BENCH=1 RESNET=1 bash tools/gpu_ab_env.sh r05v ORION_MAC_ROWS 0 1
