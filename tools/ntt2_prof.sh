# GPU: per-pass kernel times of the two-pass NTT (rocprofv3 kernel trace) at N=2^15
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ntt2prof
export TMPDIR=/tmp JOBS=4096
for k in f64 int; do
  KINDS=$k ORION_NTT_IMPL=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ntt2prof/$k -o run --output-format csv -- python tools/ntt_bench.py > gpurun_out/ntt2prof/$k.log 2>&1 || { tail -20 gpurun_out/ntt2prof/$k.log; exit 1; }
  grep -E "us/launch" gpurun_out/ntt2prof/$k.log
  f=$(find gpurun_out/ntt2prof/$k -name "*kernel_stats.csv" | head -1)
  python -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows:
    if 'ntt' in r['Name']: print('$k', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg')
"
done
