# r04s: LoLA B=64 with the radix-4 latency kernels taking more of the
# partial-round launches (ORION_NTT2S_BELOW 128 / 256 / 512)
set -o pipefail
cd $GRAFT_REPO_ROOT
PARITY=0 NTT=0 BENCH=2 KPROF=0 RESNET=0 bash tools/ab.sh r04s env ORION_NTT2S_BELOW 128 256 512
