# GPU: parity tests, then NTT microbench of the product build vs variants.
# usage: bash tools/ntt_variants.sh name1 name2 ...   (orion_amd/_build/liborion_hip_<name>.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export JOBS=${JOBS:-1024}
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/pytest_gpu.txt
timeout -k 10 200 python tools/ntt_bench.py > gpurun_out/var_base.txt 2>&1 || exit 1
echo "== base"; cat gpurun_out/var_base.txt
for v in "$@"; do
  ORION_LIB=orion_amd/_build/liborion_hip_$v.so TAG=_$v timeout -k 10 200 python tools/ntt_bench.py > gpurun_out/var_$v.txt 2>&1 || exit 1
  echo "== $v"; cat gpurun_out/var_$v.txt
done
