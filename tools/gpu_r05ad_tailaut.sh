# GPU: the rotations' scatter-store ModDown NTTs on the two-pass kernels
# (ORION_NTT2_TAIL_AUT 0 / 1): parity with the switch on, then the B=64 line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ORION_NTT2_TAIL_AUT=1 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "lola or rotate or deferral or peer or linear or mlp" > gpurun_out/pytest_r05ad_aut1.log 2>&1 || { tail -30 gpurun_out/pytest_r05ad_aut1.log; exit 1; }
tail -1 gpurun_out/pytest_r05ad_aut1.log
PK=none B1=0 BENCH=3 RESNET=0 KPROF=0 bash tools/gpu_ab_env.sh r05ad ORION_NTT2_TAIL_AUT 0 1
