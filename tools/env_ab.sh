# A/B of one runtime switch on the LoLA bench: VAR=<env name> bash tools/env_ab.sh v1 v2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do for v in "$@"; do
  env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/envab_$v.log 2>&1 || { echo "bench failed at $v"; tail -5 gpurun_out/envab_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/envab_$v.log').read().strip().splitlines()[-1]); print('$VAR=$v', d['value'], d['ms_per_step'], d['roofline']['frac'], d['batch1']['ms_per_image'], d['kernel_ms_per_step'])"
done; done
