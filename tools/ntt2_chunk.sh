# GPU: two-pass NTT with chunked, reused scratch (Infinity Cache residency) vs one-pass
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export JOBS=4096
ORION_NTT_IMPL=2 ORION_NTT2_CHUNK=256 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "ntt or rescale or mul_relin" --timeout 120 --timeout-method thread > gpurun_out/pytest_chunk.txt 2>&1 || { tail -30 gpurun_out/pytest_chunk.txt; exit 1; }
tail -1 gpurun_out/pytest_chunk.txt
echo "== one-pass"; KINDS=f64,int timeout -k 10 200 python tools/ntt_bench.py 2>&1 | grep us/launch
for c in 0 128 256 512 1024; do
  echo "== two-pass chunk $c"
  ORION_NTT_IMPL=2 ORION_NTT2_CHUNK=$c KINDS=f64,int timeout -k 10 200 python tools/ntt_bench.py 2>&1 | grep us/launch || exit 1
done
