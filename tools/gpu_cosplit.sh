cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "ntt_roundtrip or ntt_one_pass" -m gpu > gpurun_out/cs_parity0.log 2>&1 || { tail -20 gpurun_out/cs_parity0.log; exit 1; }
ORION_NTT_COSPLIT=0.5 ORION_NTT_COSPLIT_MIN=200 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "ntt_roundtrip or ntt_one_pass" -m gpu > gpurun_out/cs_parity.log 2>&1 || { tail -20 gpurun_out/cs_parity.log; exit 1; }
tail -2 gpurun_out/cs_parity.log
for cfg in "0 2" "0.000001 2" "0.3 2" "0.5 2" "0.25 3" "0.6 1"; do
  set -- $cfg
  echo "== cosplit $1 q $2"
  ORION_NTT_COSPLIT=$1 ORION_NTT_COSPLIT_Q=$2 JOBS=1024,4096 timeout -k 10 200 python -u tools/ntt_bench.py 2>&1 | grep -v "^\[" || exit 1
done
