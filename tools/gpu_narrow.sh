# GPU: full -m gpu suite, ResNet-20 N=2^16 (batch 1) and the LoLA bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-nar}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/pytest_$TAG.log | head; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
WORKLOAD=resnet20_n16 BATCH=1 timeout -k 10 400 python -u tools/resnet_bench.py > gpurun_out/resnet_n16_$TAG.log 2>&1 || { tail -20 gpurun_out/resnet_n16_$TAG.log; exit 1; }
grep workload gpurun_out/resnet_n16_$TAG.log
WORKLOAD=resnet20_n13 BATCH=1,8 timeout -k 10 400 python -u tools/resnet_bench.py > gpurun_out/resnet_n13_$TAG.log 2>&1 || { tail -20 gpurun_out/resnet_n13_$TAG.log; exit 1; }
grep workload gpurun_out/resnet_n13_$TAG.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'])" gpurun_out/bench_$TAG.log
