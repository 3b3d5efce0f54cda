# r04x: ResNet-20 N=2^16 profile (kernel trace + SQ pass) and the batch-1
# kernel trace at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_resnet_prof.sh r04x || exit 1
bash tools/gpu_b1_prof.sh r04x
