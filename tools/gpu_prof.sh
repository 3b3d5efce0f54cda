# rocprofv3 passes over the bench command (kernel trace + separate PMC passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01}
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-extras"
rm -f gpurun_out/prof_$TAG/ntt_log_*.txt; mkdir -p gpurun_out/prof_$TAG
ORION_NTT_LOG=gpurun_out/prof_$TAG/ntt_log_kt.txt timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o kt --output-format csv -- python bench.py $ARGS > gpurun_out/prof_${TAG}_kt.log 2>&1 || { echo "kt failed"; tail -20 gpurun_out/prof_${TAG}_kt.log; exit 1; }
echo "kt ok"
ORION_NTT_LOG=gpurun_out/prof_$TAG/ntt_log_pmc_fetch.txt timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "ntt" -d gpurun_out/prof_$TAG -o pmc_fetch --output-format csv -- python bench.py $ARGS > gpurun_out/prof_${TAG}_fetch.log 2>&1 || { echo "fetch failed"; tail -20 gpurun_out/prof_${TAG}_fetch.log; exit 1; }
echo "fetch ok"
ORION_NTT_LOG=gpurun_out/prof_$TAG/ntt_log_pmc_write.txt timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "ntt" -d gpurun_out/prof_$TAG -o pmc_write --output-format csv -- python bench.py $ARGS > gpurun_out/prof_${TAG}_write.log 2>&1 || { echo "write failed"; tail -20 gpurun_out/prof_${TAG}_write.log; exit 1; }
echo "write ok"
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-include-regex "ntt|lt_bsgs|lt_giant|basis_ext|ks_mac|modup_all" -d gpurun_out/prof_$TAG -o pmc_sq --output-format csv -- python bench.py $ARGS > gpurun_out/prof_${TAG}_sq.log 2>&1 || { echo "sq failed"; tail -20 gpurun_out/prof_${TAG}_sq.log; exit 1; }
echo "sq ok"

# summarise on the box (only gpurun_out/ comes back, <= 64 MiB): the summaries go to
# gpurun_out/summ_<tag>/ (copied into profiles/ afterwards), the raw traces are dropped
python tools/pmc_summary.py $TAG gpurun_out/summ_$TAG && rm -f gpurun_out/prof_$TAG/*_kernel_trace.csv gpurun_out/prof_$TAG/*_counter_collection.csv
