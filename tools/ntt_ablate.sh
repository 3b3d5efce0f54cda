# timing-only NTT ablation: full kernel vs no-compute / no-exchange / memory-only
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export JOBS=1024
timeout -k 10 200 python tools/ntt_bench.py > gpurun_out/abl0.txt 2>&1 || exit 1
for k in 1 2 3; do
  ORION_LIB=orion_amd/_build/liborion_hip_abl$k.so TAG=_abl$k timeout -k 10 200 python tools/ntt_bench.py > gpurun_out/abl$k.txt 2>&1 || exit 1
done
grep -h "jobs" gpurun_out/abl0.txt gpurun_out/abl1.txt gpurun_out/abl2.txt gpurun_out/abl3.txt
