# one GPU call: shader clock under load + NTT at a full and a half persistent grid
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02h}
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench/clock_probe > gpurun_out/clock_$TAG.txt 2>&1 || { echo "probe failed"; tail gpurun_out/clock_$TAG.txt; exit 1; }
cat gpurun_out/clock_$TAG.txt
for gr in 256 128 64; do
  echo "== grid $gr"
  ORION_NTT_GRID=$gr JOBS=1024 KINDS=f64,int TAG=_g$gr timeout -k 10 120 python tools/ntt_bench.py 2>&1 | grep -v amdgpu.ids || { echo "ntt_bench failed"; exit 1; }
done
