# r04i: the whole GPU suite (basis-extension target records, modup_all
# pointer walk, float64 narrow reduction), then the ResNet-20 N=2^16 profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r04i.log 2>&1 || { tail -30 gpurun_out/pytest_r04i.log; exit 1; }
tail -1 gpurun_out/pytest_r04i.log
bash tools/gpu_resnet_prof.sh r04i
