# A/B: plain forward launches with a partial last round on the two-pass kernels (ORION_NTT2_TAIL_FWD)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do for f in ${FS:-0 1}; do
  ORION_NTT2_TAIL_FWD=$f timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/tailfwd_$f.log 2>&1 || { echo "bench failed at $f"; tail -5 gpurun_out/tailfwd_$f.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/tailfwd_$f.log').read().strip().splitlines()[-1]); print('fwd=$f', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernel_ms_per_step']['ntt_fwd'], d['kernel_ms_per_step']['ntt_inv'])"
done; done
