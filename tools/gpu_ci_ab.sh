# one GPU call: mem_split ubench, headline bench, CI workloads native vs the r01/r02 emulation (2N Standard ring)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02f}
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench/mem_split > gpurun_out/mem_split_$TAG.txt 2>&1 || { echo "ubench failed"; tail gpurun_out/mem_split_$TAG.txt; exit 1; }
cat gpurun_out/mem_split_$TAG.txt
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -c 700 gpurun_out/bench_$TAG.log; echo
for w in lola_n13_ci mlp_n13_ci; do
  for v in native emu; do
    if [ $v = emu ]; then L=orion_amd/_build/liborion_hip_emu.so; else L=orion_amd/liborion_hip.so; fi
    ORION_LIB=$L timeout -k 10 300 python bench.py --workload $w --batch 64 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ci_${w}_${v}_$TAG.log 2>&1 || { echo "ci bench $w $v failed"; tail -20 gpurun_out/ci_${w}_${v}_$TAG.log; exit 1; }
    echo "$w $v: $(tail -1 gpurun_out/ci_${w}_${v}_$TAG.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"], "ms/step", d.get("check"))')"
  done
done
