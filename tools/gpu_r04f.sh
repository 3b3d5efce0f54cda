set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B1=2 BENCH=2 KPROF=1 RESNET=0 bash tools/gpu_ab_env.sh r04f ORION_LT_SPLIT_KEYS 0 1 || exit 1
PK="ntt or lola" B1=2 BENCH=1 KPROF=0 RESNET=1 bash tools/gpu_ab_env.sh r04g ORION_NTT2S_BELOW 128 256 1024 || exit 1
