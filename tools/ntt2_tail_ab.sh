# A/B of the partial-round rule (ORION_NTT2_TAIL_EFF; 0 = off) on the LoLA bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do for e in ${@:-0 0.8 0.9 0.95}; do
  ORION_NTT2_TAIL_EFF=$e timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/tail_$e.log 2>&1 || { echo "bench failed at $e"; tail -5 gpurun_out/tail_$e.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/tail_$e.log').read().strip().splitlines()[-1]); print('eff=$e', d['value'], d['ms_per_step'], d['roofline']['frac'], d['batch1']['ms_per_image'], d['kernel_ms_per_step']['ntt_fwd'], d['kernel_ms_per_step']['ntt_inv'])"
done; done
