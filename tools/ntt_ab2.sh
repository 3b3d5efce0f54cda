# GPU: product library (parity subset + NTT microbench + bench) against
# timing-only variants orion_amd/_build/liborion_hip_<V>.so named in $VARS
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ops.py -x -q -m gpu -k "ntt or lola_n15_matches or mul_relin or rescale or linear or conjugate or n16" --timeout 120 --timeout-method thread > gpurun_out/pytest_ab2.txt 2>&1 || { tail -30 gpurun_out/pytest_ab2.txt; exit 1; }
tail -1 gpurun_out/pytest_ab2.txt
for v in base $VARS; do
  if [ $v = base ]; then L=orion_amd/liborion_hip.so; else L=orion_amd/_build/liborion_hip_$v.so; fi
  ORION_LIB=$L KINDS=${KINDS:-f64,int,mix} JOBS=${JOBS:-192,384,640,4096} timeout -k 10 200 python tools/ntt_bench.py > gpurun_out/nb_$v.txt 2>&1 || { tail -5 gpurun_out/nb_$v.txt; exit 1; }
  echo "== $v"; cat gpurun_out/nb_$v.txt
done
for rep in 1 2; do for v in base $VARS; do
  if [ $v = base ]; then L=orion_amd/liborion_hip.so; else L=orion_amd/_build/liborion_hip_$v.so; fi
  ORION_LIB=$L timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$v.txt 2>&1 || { tail -5 gpurun_out/bench_$v.txt; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_$v.txt').read().strip().splitlines()[-1]); print('$v', d['value'], 'img/s', d['roofline']['avg_launch_us'], 'us/NTT', d['roofline']['frac'], d['kernel_ms_per_step']['ntt_fwd'], d['kernel_ms_per_step']['ntt_inv'])"
done; done
