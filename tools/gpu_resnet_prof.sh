# GPU: rocprofv3 passes over one ResNet-20 N=2^16 inference (tools/resnet_bench.py, batch 1):
# kernel trace + stats, then one SQ/GRBM counter pass (VALU busy, wait, SALU:VALU) over every
# kernel (no include filter: tools/pmc_summary.py --resnet cuts both passes to the timed
# inference by dispatch position, between the PROF_MARK idle gaps of the kernel trace).  usage: bash tools/gpu_resnet_prof.sh TAG   -> gpurun_out/prof_rn16_TAG/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r03}
D=gpurun_out/prof_rn16_$TAG
mkdir -p $D
PROF_MARK=1 WORKLOAD=resnet20_n16 BATCH=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D -o kt --output-format csv -- python -u tools/resnet_bench.py > ${D}_kt.log 2>&1 || { tail -20 ${D}_kt.log; exit 1; }
tail -1 ${D}_kt.log
[ "${2:-}" = "nopmc" ] && { python tools/pmc_summary.py --resnet $TAG gpurun_out/summ_$TAG; rm -f ${D}/*_kernel_trace.csv; exit 0; }
PROF_MARK=1 WORKLOAD=resnet20_n16 BATCH=1 timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $D -o pmc_sq --output-format csv -- python -u tools/resnet_bench.py > ${D}_sq.log 2>&1 || { tail -20 ${D}_sq.log; exit 1; }
tail -1 ${D}_sq.log
python tools/pmc_summary.py --resnet $TAG gpurun_out/summ_$TAG && rm -f ${D}/*_kernel_trace.csv ${D}/*_counter_collection.csv
