# GPU: full -m gpu suite, NTT microbench and the LoLA bench (no CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-chk}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/pytest_$TAG.log | head; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
JOBS=1024,4096 timeout -k 10 200 python -u tools/ntt_bench.py > gpurun_out/nb_$TAG.txt 2>&1 || { tail -20 gpurun_out/nb_$TAG.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/nb_$TAG.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_$i.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_$i.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['kernel_ms_per_step']['ntt_fwd'], d['kernel_ms_per_step']['ntt_inv'])" gpurun_out/bench_${TAG}_$i.log
done
