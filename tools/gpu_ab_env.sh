# GPU A/B of one runtime switch (or of library builds), one gpurun call:
#   bash tools/gpu_ab_env.sh TAG VAR A B ...          VAR=A, VAR=B, ... on the product library
#   MODE=lib bash tools/gpu_ab_env.sh TAG - V1 V2 ... library variants (tools/build_ablation.py;
#                                                     V = product: the in-tree library)
# Steps (env knobs, defaults in brackets):
#   PK    [ntt or linear or ...]  pytest -k selection of the GPU suite run first on the
#                                 defaults; "all": the whole suite; "none": skipped
#   B1    [2]   batch-1 bench repetitions per value (B1_STEPS [20], B1_WARMUP [3]); 0: none
#   BENCH [2], KPROF [0], RESNET [1]: LoLA B=64 bench repetitions, a rocprofv3 kernel trace
#                                 per value, ResNet-20 N=2^16 per value (tools/ab.sh)
# Output: gpurun_out/ab_<TAG>_* and one summary line per run on stdout.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:?tag}; VAR=${2:?var}; shift 2
MODE=${MODE:-env}
mkdir -p gpurun_out
PK=${PK:-ntt or linear or lola or mlp or rotate or deep or rescale or mul_relin or bootstrap or resnet20_n13_prefix or n16}
if [ "$PK" != none ]; then
  sel=(-k "$PK"); [ "$PK" = all ] && sel=()
  timeout -k 10 700 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests "${sel[@]}" > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -1 gpurun_out/pytest_$TAG.log
fi
with() {  # with VALUE cmd...: the value's switch or library applied to one command
  local v=$1; shift
  if [ "$MODE" = lib ]; then
    local lib=orion_amd/liborion_hip.so; [ "$v" != product ] && lib=orion_amd/_build/liborion_hip_$v.so
    ORION_LIB=$lib "$@"
  else
    env "$VAR=$v" "$@"
  fi
}
for r in $(seq 1 ${B1:-2}); do
  for v in "$@"; do
    with $v timeout -k 10 300 python bench.py --batch 1 --steps ${B1_STEPS:-20} --warmup ${B1_WARMUP:-3} --no-cpu-baseline --no-extras > gpurun_out/ab_${TAG}_b1_${v}_$r.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_b1_${v}_$r.log; exit 1; }
    echo "$v batch1 $r: $(tail -1 gpurun_out/ab_${TAG}_b1_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/image")')"
  done
done
if [ "$MODE" = lib ]; then
  PARITY=0 NTT=0 BENCH=${BENCH:-2} KPROF=${KPROF:-0} RESNET=${RESNET:-1} bash tools/ab.sh $TAG lib "$@"
else
  PARITY=0 NTT=0 BENCH=${BENCH:-2} KPROF=${KPROF:-0} RESNET=${RESNET:-1} bash tools/ab.sh $TAG env $VAR "$@"
fi
