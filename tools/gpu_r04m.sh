# r04m (one box): lt_bsgs without per-slot branches (LT_DENSE: unused plan
# slots point at a zero diagonal) vs the branchy build (parity, LoLA bench,
# kernel trace, ResNet); then ResNet-20 N=2^16 with the basis-extension target
# modes and the INTT -> prologue-NTT fusion (MODES/IFUSE = 0/0, 1/0, 1/1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PARITY=1 NTT=0 BENCH=2 KPROF=1 RESNET=1 bash tools/ab.sh r04m lib product sparse || exit 1
for v in 00 10 11; do
  ORION_BEXT_MODES=${v:0:1} ORION_NTT_IFUSE=${v:1:1} WORKLOAD=resnet20_n16 BATCH=1 timeout -k 10 300 python -u tools/resnet_bench.py > gpurun_out/r04m_resnet_$v.log 2>&1 || { tail -20 gpurun_out/r04m_resnet_$v.log; exit 1; }
  echo "MODES/IFUSE=$v: $(grep workload gpurun_out/r04m_resnet_$v.log | tail -1 | cut -c90-160)"
done
