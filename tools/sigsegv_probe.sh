# The round-2 host SIGSEGV (profiles/r03a_sigsegv_probe.txt): the bench with its
# hipGraph extras under a rocprofv3 PMC pass, with /proc/self/maps dumped
# before the extras (bench.py ORION_DUMP_MAPS) so that the PCs of the crash
# report resolve to library + offset.  Run it as the LAST GPU step of a call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r03a}
mkdir -p gpurun_out/segv_$TAG
ORION_BENCH_STAGES=1 ORION_DUMP_MAPS=gpurun_out/segv_$TAG/maps timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE \
  --kernel-include-regex "ntt" -d gpurun_out/segv_$TAG -o pmc_fetch --output-format csv -- \
  python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/segv_$TAG/extras.log 2>&1
rc=$?
echo "pmc + extras rc=$rc"
tail -40 gpurun_out/segv_$TAG/extras.log
exit $rc
