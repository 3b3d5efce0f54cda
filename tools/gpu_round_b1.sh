# one GPU call: the round profile (tools/gpu_round.sh) and the batch-1 kernel
# trace (tools/gpu_b1_prof.sh) with its per-pass summary
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
bash tools/gpu_round.sh $TAG || exit 1
bash tools/gpu_b1_prof.sh $TAG > gpurun_out/prof_b1_${TAG}_stats.txt 2>&1 || { tail -20 gpurun_out/prof_b1_${TAG}_stats.txt; exit 1; }
f=$(find gpurun_out/prof_b1_$TAG -name "b1_kernel_trace.csv" | head -1)
python tools/b1_trace_summ.py "$f" 20 > gpurun_out/prof_b1_${TAG}_trace_summary.txt && cat gpurun_out/prof_b1_${TAG}_trace_summary.txt
