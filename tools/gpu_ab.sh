# GPU A/B of library variants (ORION_LIB): GPU suite on the product library,
# LT parity tests on each variant, then alternating LoLA bench runs.
# usage: bash tools/gpu_ab.sh TAG variant1 variant2 ...  (orion_amd/_build/liborion_hip_<v>.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/pytest_$TAG.log | head; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for v in "$@"; do
  ORION_LIB=orion_amd/_build/liborion_hip_$v.so timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "linear or lola or mlp or rotate or deep or bootstrap" --timeout 200 --timeout-method thread > gpurun_out/pytest_${TAG}_$v.log 2>&1 || { echo "variant $v failed"; tail -20 gpurun_out/pytest_${TAG}_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/pytest_${TAG}_$v.log)"
done
for rep in 1 2; do
  for v in product "$@"; do
    lib=orion_amd/liborion_hip.so; [ $v != product ] && lib=orion_amd/_build/liborion_hip_$v.so
    ORION_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras > gpurun_out/bench_${TAG}_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_${v}_$rep.log; exit 1; }
    echo "$v $rep: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])" gpurun_out/bench_${TAG}_${v}_$rep.log)"
  done
done
# optional: ResNet-20 N=2^16 batch 1 per library (RESNET=1)
if [ "${RESNET:-0}" = 1 ]; then
  for v in product "$@"; do
    lib=orion_amd/liborion_hip.so; [ $v != product ] && lib=orion_amd/_build/liborion_hip_$v.so
    ORION_LIB=$lib WORKLOAD=resnet20_n16 BATCH=1 timeout -k 10 400 python -u tools/resnet_bench.py > gpurun_out/resnet_${TAG}_$v.log 2>&1 || { tail -20 gpurun_out/resnet_${TAG}_$v.log; exit 1; }
    echo "$v resnet: $(grep workload gpurun_out/resnet_${TAG}_$v.log | tail -1 | cut -c1-200)"
  done
fi
