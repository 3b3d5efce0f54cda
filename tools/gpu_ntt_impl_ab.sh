# NTT microbenchmark: one-pass (ORION_NTT_IMPL=1) vs two-pass (2) kernels per modulus class
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r03}
mkdir -p gpurun_out
export JOBS=${JOBS:-256,1024,4096} KINDS=${KINDS:-f64,int,mix}
for impl in 1 2; do
  ORION_NTT_IMPL=$impl ORION_NTT2_TAIL_EFF=0 TAG=_impl$impl timeout -k 10 200 python tools/ntt_bench.py > gpurun_out/nb_impl${impl}_$TAG.txt 2>&1 || { tail -20 gpurun_out/nb_impl${impl}_$TAG.txt; exit 1; }
  echo "== ORION_NTT_IMPL=$impl"; cat gpurun_out/nb_impl${impl}_$TAG.txt
done
