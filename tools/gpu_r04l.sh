# r04l: ResNet-20 N=2^16 on one box: basis-extension target modes and the
# INTT -> prologue-NTT fusion, alternating (MODES/IFUSE = 0/0, 1/0, 1/1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in 00 10 11; do
    ORION_BEXT_MODES=${v:0:1} ORION_NTT_IFUSE=${v:1:1} WORKLOAD=resnet20_n16 BATCH=1 timeout -k 10 300 python -u tools/resnet_bench.py > gpurun_out/r04l_resnet_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/r04l_resnet_${v}_$rep.log; exit 1; }
    echo "MODES/IFUSE=$v rep $rep: $(grep workload gpurun_out/r04l_resnet_${v}_$rep.log | tail -1 | cut -c90-160)"
  done
done
