# GPU: parity subset on the defaults, then an A/B of one runtime switch:
#   bash tools/gpu_ab_env.sh TAG VAR A B ...
# per value: LoLA bench (BENCH reps), batch-1 bench (stream, B1 reps), ResNet-20 N=2^16 (RESNET=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:?tag}; VAR=${2:?var}; shift 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests -k "${PK:-ntt or linear or lola or mlp or rotate or deep or rescale or mul_relin or bootstrap or resnet20_n13_prefix or n16}" > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for v in "$@"; do
  for r in $(seq 1 ${B1:-2}); do
    env $VAR=$v timeout -k 10 200 python bench.py --batch 1 --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/ab_${TAG}_b1_${v}_$r.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_b1_${v}_$r.log; exit 1; }
    echo "$VAR=$v batch1 $r: $(tail -1 gpurun_out/ab_${TAG}_b1_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/image")')"
  done
done
PARITY=0 NTT=0 BENCH=${BENCH:-2} KPROF=${KPROF:-0} RESNET=${RESNET:-1} bash tools/ab.sh $TAG env $VAR "$@"
