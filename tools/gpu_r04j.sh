# r04j: basis-extension target modes (BEXT_WT / BEXT_NT): parity, then ResNet-20
# N=2^16 and LoLA B=64 timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "basis_extension_modes or resnet or deep or bootstrap or rotate or mul_relin or lola or linear or n16" --timeout 300 --timeout-method thread > gpurun_out/pytest_r04j.log 2>&1 || { tail -30 gpurun_out/pytest_r04j.log; exit 1; }
tail -1 gpurun_out/pytest_r04j.log
WORKLOAD=resnet20_n16 BATCH=1 timeout -k 10 400 python -u tools/resnet_bench.py > gpurun_out/r04j_resnet.log 2>&1 || { tail -20 gpurun_out/r04j_resnet.log; exit 1; }
grep workload gpurun_out/r04j_resnet.log | tail -1 | cut -c1-200
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras > gpurun_out/r04j_bench.log 2>&1 || { tail -20 gpurun_out/r04j_bench.log; exit 1; }
tail -1 gpurun_out/r04j_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('kernel_ms_per_step'))"
bash tools/gpu_b1_prof.sh r04j
