# LoLA bench A/B of the two-pass tail rule: default vs full single-round launches two-pass too
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "0.9 1024" "1.01 256" "1.01 1024"; do
    set -- $cfg
    ORION_NTT2_TAIL_EFF=$1 ORION_NTT2_TAIL_MAX=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras > gpurun_out/tail_$1_$2_$rep.log 2>&1 || { echo "bench failed at $cfg"; tail -5 gpurun_out/tail_$1_$2_$rep.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('eff=$1 max=$2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernel_ms_per_step']['ntt_inv'], d['kernel_ms_per_step']['ntt_fwd'])" gpurun_out/tail_$1_$2_$rep.log
  done
done
