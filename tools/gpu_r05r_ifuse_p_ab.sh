# GPU: the shared-source fused INTT-columns kernel (ORION_NTT_IFUSE_P = 2 / 4
# groups per workgroup; 1 = one target per workgroup): the GPU suite with P=4,
# a parity subset with P=2, then batch-1 latency, the B=64 line and ResNet-20
# N=2^16 over P = 1 2 4 (SKIP_PARITY=1 skips the parity runs)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "${SKIP_PARITY:-}" ]; then
ORION_NTT_IFUSE_P=4 timeout -k 10 800 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG:-r05r}_p4.log 2>&1 || { tail -30 gpurun_out/pytest_${TAG:-r05r}_p4.log; exit 1; }
tail -1 gpurun_out/pytest_${TAG:-r05r}_p4.log
ORION_NTT_IFUSE_P=2 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "ntt or lola or mlp or resnet20_n13_prefix or n16 or deep or runtime_switch or bootstrap" > gpurun_out/pytest_${TAG:-r05r}_p2.log 2>&1 || { tail -30 gpurun_out/pytest_${TAG:-r05r}_p2.log; exit 1; }
tail -1 gpurun_out/pytest_${TAG:-r05r}_p2.log
fi
PK=none B1=2 BENCH=1 RESNET=1 bash tools/gpu_ab_env.sh ${TAG:-r05r} ORION_NTT_IFUSE_P 1 2 4
# diagnosis: ResNet-20 N=2^16 at batch 4 (r05q: "Bootstrap: modraise failed")
WORKLOAD=resnet20_n16 BATCH=4 AMD_LOG_LEVEL=1 timeout -k 10 300 python -u tools/resnet_bench.py > gpurun_out/${TAG:-r05r}_resnet_b4.jsonl 2> gpurun_out/${TAG:-r05r}_resnet_b4.err; echo "resnet batch 4 rc=$?"; tail -5 gpurun_out/${TAG:-r05r}_resnet_b4.err
