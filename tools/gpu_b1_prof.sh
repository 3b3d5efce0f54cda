# GPU: kernel trace of the batch-1 LoLA stream (BASELINE configs[2]):
#   bash tools/gpu_b1_prof.sh TAG  -> gpurun_out/prof_b1_TAG/, summary on stdout
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:?tag}
D=gpurun_out/prof_b1_$TAG
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o b1 --output-format csv -- python bench.py --batch 1 --steps 20 --warmup 3 --no-cpu-baseline --no-extras > ${D}.log 2>&1 || { tail -20 ${D}.log; exit 1; }
tail -1 ${D}.log
f=$(find $D -name "b1_kernel_stats.csv" | head -1)
python tools/rocpd_stats.py --csv "$f" 25
