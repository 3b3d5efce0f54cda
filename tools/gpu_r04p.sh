# r04p: basis-extension target modes with the source pieces kept in the target
# loop (88-90 VGPRs, 5 waves per SIMD, instead of 170-202 and 2): parity, then
# ResNet-20 N=2^16 with the modes off/on (same box), then a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "basis_extension_modes or resnet or n16 or bootstrap or deep" --timeout 300 --timeout-method thread > gpurun_out/pytest_r04p.log 2>&1 || { tail -30 gpurun_out/pytest_r04p.log; exit 1; }
tail -1 gpurun_out/pytest_r04p.log
for rep in 1 2; do
  for v in 0 1; do
    ORION_BEXT_MODES=$v WORKLOAD=resnet20_n16 BATCH=1 timeout -k 10 300 python -u tools/resnet_bench.py > gpurun_out/r04p_resnet_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/r04p_resnet_${v}_$rep.log; exit 1; }
    echo "MODES=$v rep $rep: $(grep workload gpurun_out/r04p_resnet_${v}_$rep.log | tail -1 | cut -c90-160)"
  done
done
bash tools/gpu_resnet_prof.sh r04p nopmc
