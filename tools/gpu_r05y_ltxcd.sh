# GPU: XCD-aware workgroup order in lt_bsgs / lt_giant (ORION_LT_XCD 0 / 1):
# LT parity with the switch on, then batch 1 / B=64 / ResNet-20 N=2^16
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ORION_LT_XCD=1 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "linear or lola or resnet20_n13_prefix or n16 or bootstrap or mlp" > gpurun_out/pytest_r05y_xcd1.log 2>&1 || { tail -30 gpurun_out/pytest_r05y_xcd1.log; exit 1; }
tail -1 gpurun_out/pytest_r05y_xcd1.log
PK=none B1=1 BENCH=2 RESNET=1 bash tools/gpu_ab_env.sh r05y ORION_LT_XCD 0 1
