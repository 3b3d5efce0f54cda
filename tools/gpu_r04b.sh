# round-4 A/B of the fused basis extension (NTT_PRO_BEXT): LoLA bench x2,
# kernel profiles, ResNet-20 N=2^16, batch-1 bench (stream launches) per setting
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r04b}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests -k "ntt or linear or lola or mlp or rotate or deep or rescale or mul_relin or bootstrap or resnet20_n13_prefix" > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
PARITY=0 NTT=0 BENCH=2 KPROF=1 RESNET=${RESNET:-1} bash tools/ab.sh $TAG env ORION_BEXT_FUSE 0 1 || exit 1
for v in 0 1; do for r in 1 2; do
  ORION_BEXT_FUSE=$v timeout -k 10 200 python bench.py --batch 1 --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/ab_${TAG}_b1_${v}_$r.log 2>&1 || exit 1
  echo "fuse=$v batch1 run $r: $(tail -1 gpurun_out/ab_${TAG}_b1_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/image")')"
done; done
if [ "${FULLBENCH:-0}" = 1 ]; then
  timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
  tail -1 gpurun_out/bench_$TAG.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("full bench:", d["value"], d["ms_per_step"], d["roofline"]["frac"], d.get("batch1"), d.get("kernel_ms_per_step"))'
fi
