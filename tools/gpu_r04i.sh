# r04i: parity subset after the split-key removal, then the ResNet-20 N=2^16 profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "linear or lola or bootstrap or rotate" --timeout 200 --timeout-method thread > gpurun_out/pytest_r04i.log 2>&1 || { tail -30 gpurun_out/pytest_r04i.log; exit 1; }
tail -1 gpurun_out/pytest_r04i.log
bash tools/gpu_resnet_prof.sh r04i
