# GPU A/B harness (one gpurun call): the variants below are measured on the same box,
# alternating, so box-to-box noise cancels.
#
#   bash tools/ab.sh TAG lib  V1 V2 ...        library variants orion_amd/_build/liborion_hip_<V>.so
#                                              (V = product: the in-tree orion_amd/liborion_hip.so)
#   bash tools/ab.sh TAG env  VAR A B ...      one runtime switch VAR=A, VAR=B, ... on the product library
#
# Steps per variant (env knobs, defaults in brackets):
#   PARITY [1]  GPU parity subset on the variant (NTT, key switch, LT, replays)
#   NTT    [1]  tools/ntt_bench.py (JOBS [256,1024,4096], KINDS [f64,int,mix])
#   BENCH  [2]  LoLA bench.py repetitions (no CPU baseline, no extras)
#   RESNET [0]  ResNet-20 N=2^16 batch 1 (tools/resnet_bench.py)
#   KPROF  [0]  rocprofv3 --kernel-trace --stats of one short bench per variant
# Output: gpurun_out/ab_<TAG>_* and one summary line per run on stdout.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:?tag}; MODE=${2:?lib or env}; shift 2
if [ "$MODE" = env ]; then VAR=${1:?variable}; shift; fi
mkdir -p gpurun_out
O=gpurun_out/ab_$TAG
run_env() {  # run_env VARIANT cmd... : the variant's library / switch applied to one command
  local v=$1; shift
  if [ "$MODE" = lib ]; then
    local lib=orion_amd/liborion_hip.so; [ "$v" != product ] && lib=orion_amd/_build/liborion_hip_$v.so
    ORION_LIB=$lib "$@"
  else
    env "$VAR=$v" "$@"
  fi
}
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], 'img/s', d['ms_per_step'], 'ms/step, NTT frac', d['roofline']['frac'], d['roofline'].get('avg_launch_us'), 'us', d.get('kernel_ms_per_step'))" "$1"; }
if [ "${PARITY:-1}" = 1 ]; then
  for v in "$@"; do
    run_env $v timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "ntt or linear or lola or mlp or rotate or deep or rescale or mul_relin or bootstrap" --timeout 200 --timeout-method thread > ${O}_pytest_$v.log 2>&1 || { echo "variant $v failed parity"; tail -30 ${O}_pytest_$v.log; exit 1; }
    echo "$v parity: $(tail -1 ${O}_pytest_$v.log)"
  done
fi
if [ "${NTT:-1}" = 1 ]; then
  for v in "$@"; do
    run_env $v env JOBS=${JOBS:-256,1024,4096} KINDS=${KINDS:-f64,int,mix} timeout -k 10 300 python tools/ntt_bench.py > ${O}_ntt_$v.txt 2>&1 || { echo "ntt_bench $v failed"; tail -20 ${O}_ntt_$v.txt; exit 1; }
    echo "== $v ntt_bench"; grep jobs ${O}_ntt_$v.txt
  done
fi
for rep in $(seq 1 ${BENCH:-2}); do
  for v in "$@"; do
    run_env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras > ${O}_bench_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -20 ${O}_bench_${v}_$rep.log; exit 1; }
    echo "$v bench $rep: $(summ ${O}_bench_${v}_$rep.log)"
  done
done
if [ "${RESNET:-0}" = 1 ]; then
  for v in "$@"; do
    run_env $v env WORKLOAD=resnet20_n16 BATCH=1 timeout -k 10 400 python -u tools/resnet_bench.py > ${O}_resnet_$v.log 2>&1 || { echo "resnet $v failed"; tail -20 ${O}_resnet_$v.log; exit 1; }
    echo "$v resnet: $(grep workload ${O}_resnet_$v.log | tail -1 | cut -c1-220)"
  done
fi
if [ "${KPROF:-0}" = 1 ]; then
  for v in "$@"; do
    run_env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_kprof -o $v --output-format csv -- python bench.py --no-cpu-baseline --no-extras --steps 5 --warmup 2 > ${O}_kprof_$v.log 2>&1 || { echo "kprof $v failed"; tail -20 ${O}_kprof_$v.log; exit 1; }
    f=$(find ${O}_kprof -name "${v}_kernel_stats.csv" | head -1)
    python tools/rocpd_stats.py --csv "$f" 10 | sed "s/^/$v  /"
  done
fi
