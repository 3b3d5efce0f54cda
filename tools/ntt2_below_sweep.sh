# A/B of the one-pass/two-pass switch point at N=2^15 (ORION_NTT2_BELOW,
# limb-transforms per launch) on the LoLA bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in ${@:-128 400 700 1000 2000}; do
  ORION_NTT2_BELOW=$b timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/below_$b.log 2>&1 || { echo "bench failed at $b"; tail -5 gpurun_out/below_$b.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/below_$b.log').read().strip().splitlines()[-1]); print($b, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['kernel_ms_per_step']['ntt_fwd'], d['kernel_ms_per_step']['ntt_inv'])"
done
