set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/_ubench_valu > gpurun_out/ubench_valu_r05i.txt 2>&1 && cat gpurun_out/ubench_valu_r05i.txt || exit 1
for r in 1 2; do
  for cfg in "2 128" "4 128" "2 257"; do
    set -- $cfg
    o=gpurun_out/ab_r05i_p$1_b$2_$r.log
    ORION_NTT2_BELOW=$2 timeout -k 10 300 python bench.py --pipelines $1 --no-cpu-baseline --no-extras > $o 2>&1 || { tail -20 $o; exit 1; }
    echo "P=$1 NTT2_BELOW=$2 rep $r: $(tail -1 $o | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "img/s", d["ms_per_step"], "ms; frac", d["roofline"]["frac"], d["kernel_ms_per_step"])')"
  done
done
