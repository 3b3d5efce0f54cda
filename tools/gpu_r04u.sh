# r04u: lt_giant reducing once per giant on moduli up to 2^60 (LT_GIANT_ACC8,
# product) vs once per chunk of digits (noacc8g build), one box
set -o pipefail
cd $GRAFT_REPO_ROOT
PARITY=1 NTT=0 BENCH=2 KPROF=1 RESNET=1 bash tools/ab.sh r04u lib product noacc8g
