# r04t: one-pass launches with a partial last round split into whole rounds
# (one-pass) + the partial round (two-pass kernels), ORION_NTT_TAILSPLIT 0/1:
# parity subset with it on, then LoLA B=64 bench + kernel trace per value
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ORION_NTT_TAILSPLIT=1 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "ntt or lola or linear or rescale or mul_relin or rotate" --timeout 300 --timeout-method thread > gpurun_out/pytest_r04t.log 2>&1 || { tail -30 gpurun_out/pytest_r04t.log; exit 1; }
tail -1 gpurun_out/pytest_r04t.log
PARITY=0 NTT=0 BENCH=2 KPROF=1 RESNET=0 bash tools/ab.sh r04t env ORION_NTT_TAILSPLIT 0 1
