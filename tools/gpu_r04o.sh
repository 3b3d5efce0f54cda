# r04o: batch-1 kernel trace and the ResNet-20 N=2^16 profile at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_b1_prof.sh r04o || exit 1
bash tools/gpu_resnet_prof.sh r04o
