# GPU: NTT parity tests, then the NTT microbenchmark for the product build and variants
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export JOBS=${JOBS:-1024,4096}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k ntt --timeout 120 --timeout-method thread > gpurun_out/pytest_ntt.txt 2>&1 || { tail -30 gpurun_out/pytest_ntt.txt; exit 1; }
tail -1 gpurun_out/pytest_ntt.txt
run() { tag=$1; shift; env "$@" TAG=_$tag timeout -k 10 200 python tools/ntt_bench.py > gpurun_out/nb_$tag.txt 2>&1 || exit 1; echo "== $tag"; cat gpurun_out/nb_$tag.txt; }
run base
for v in "$@"; do run $v ORION_LIB=orion_amd/_build/liborion_hip_$v.so; done
