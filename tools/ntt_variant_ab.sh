# GPU: A/B of a timing variant library (orion_amd/_build/liborion_hip_$V.so)
# against the product library on one box: NTT parity, NTT microbench, bench.py
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=${V:?variant name}
VL=orion_amd/_build/liborion_hip_$V.so
export JOBS=${JOBS:-4096}
ORION_LIB=$VL timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ops.py -x -q -m gpu -k "ntt or lola_n15_matches or mul_relin or rescale or linear" --timeout 120 --timeout-method thread > gpurun_out/pytest_$V.txt 2>&1 || { tail -30 gpurun_out/pytest_$V.txt; exit 1; }
tail -1 gpurun_out/pytest_$V.txt
for lib in base $V; do
  if [ $lib = base ]; then L=orion_amd/liborion_hip.so; else L=$VL; fi
  ORION_LIB=$L TAG=_$lib timeout -k 10 200 python tools/ntt_bench.py > gpurun_out/nb_$lib.txt 2>&1 || exit 1
  echo "== $lib"; cat gpurun_out/nb_$lib.txt
  ORION_LIB=$L timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$lib.txt 2>&1 || { tail -5 gpurun_out/bench_$lib.txt; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_$lib.txt').read().strip().splitlines()[-1]); print('$lib', d['value'], 'img/s', d['roofline']['avg_launch_us'], 'us/NTT', d['roofline']['frac'], d['kernel_ms_per_step'])"
done
