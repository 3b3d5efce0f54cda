set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ORION_NTT2_CHUNK=256 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "ntt or n16 or deep or lola or resnet20_n13_prefix" > gpurun_out/pytest_r05l_chunk256.log 2>&1 || { tail -30 gpurun_out/pytest_r05l_chunk256.log; exit 1; }
tail -1 gpurun_out/pytest_r05l_chunk256.log
PK=none B1=0 BENCH=1 RESNET=1 bash tools/gpu_ab_env.sh r05l ORION_NTT2_CHUNK 0 128 256 512
