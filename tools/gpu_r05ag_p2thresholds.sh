# GPU: two-pass thresholds under 2 peer pipelines (each launch is half the
# batch, and the other pipeline fills a launch's idle CUs): the B=64 line with
# ORION_NTT2_TAIL_EFF 0.9 (default) / 0 (partial rounds stay one-pass), then
# ORION_NTT2_BELOW 128 (default) / 64, alternating, 2 reps
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for cfg in "0.9 128" "0 128" "0.9 64"; do
    set -- $cfg
    o=gpurun_out/ab_r05ag_eff$1_below$2_$r.log
    ORION_NTT2_TAIL_EFF=$1 ORION_NTT2_BELOW=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras > $o 2>&1 || { tail -20 $o; exit 1; }
    echo "TAIL_EFF=$1 BELOW=$2 rep $r: $(tail -1 $o | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "img/s", d["ms_per_step"], "ms; solo frac", d["roofline"]["frac"], "union", d["roofline"]["concurrent"]["frac_union"])')"
  done
done
