# one GPU call: NTT stagger sweep (ntt_bench) + LoLA bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02g}
mkdir -p gpurun_out
for st in 0 1 2 3 4 6; do
  echo "== stagger $st"
  ORION_NTT_STAGGER=$st ORION_NTT_STAGGER_MIN=1 JOBS=1024,4096 KINDS=f64,mix TAG=_st$st timeout -k 10 120 python tools/ntt_bench.py > gpurun_out/ntt_st${st}_$TAG.txt 2>&1 || { echo "ntt_bench failed"; tail gpurun_out/ntt_st${st}_$TAG.txt; exit 1; }
  cat gpurun_out/ntt_st${st}_$TAG.txt
done
for st in 0 2 3; do
  ORION_NTT_STAGGER=$st timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_st${st}_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_st${st}_$TAG.log; exit 1; }
  echo "bench stagger $st: $(tail -1 gpurun_out/bench_st${st}_$TAG.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d["kernel_ms_per_step"]["ntt_fwd"], d["kernel_ms_per_step"]["ntt_inv"])')"
done
