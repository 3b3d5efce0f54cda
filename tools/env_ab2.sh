# A/B of a runtime switch: ntt_bench + bench.py (no CPU baseline) under VAR=A and VAR=B
# usage: bash tools/env_ab2.sh VAR A B TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VAR=$1; A=$2; B=$3; TAG=${4:-ab}
for v in $A $B $A $B; do
  env $VAR=$v JOBS=1024,4096 timeout -k 10 200 python tools/ntt_bench.py > gpurun_out/${TAG}_ntt_$v.txt 2>&1 || { echo "ntt_bench failed"; tail gpurun_out/${TAG}_ntt_$v.txt; exit 1; }
  env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/${TAG}_bench_$v.log 2>&1 || { echo "bench failed"; tail gpurun_out/${TAG}_bench_$v.log; exit 1; }
  echo "$VAR=$v: $(python -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_bench_$v.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['kernel_ms_per_step'])")"
done
for v in $A $B; do echo "== $VAR=$v"; grep jobs gpurun_out/${TAG}_ntt_$v.txt; done
