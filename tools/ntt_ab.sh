# GPU: NTT microbench, one-pass (impl 1) vs two-pass (impl 2), same box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export JOBS=${JOBS:-1024,4096}
ORION_NTT_IMPL=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k ntt --timeout 120 --timeout-method thread > gpurun_out/pytest_ntt2.txt 2>&1 || { tail -30 gpurun_out/pytest_ntt2.txt; exit 1; }
tail -1 gpurun_out/pytest_ntt2.txt
for impl in 1 2; do
  ORION_NTT_IMPL=$impl TAG=_impl$impl timeout -k 10 200 python tools/ntt_bench.py > gpurun_out/nb_impl$impl.txt 2>&1 || exit 1
  echo "== impl $impl"; cat gpurun_out/nb_impl$impl.txt
done
