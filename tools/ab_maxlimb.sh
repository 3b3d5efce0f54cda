set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
for lib in base lim48; do
  if [ $lib = base ]; then L=orion_amd/liborion_hip.so; else L=orion_amd/_build/liborion_hip_$lib.so; fi
  ORION_LIB=$L timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$lib.txt 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/ab_$lib.txt').read().strip().splitlines()[-1]); print('$lib', d['value'], d['kernel_ms_per_step'])"
done
done
