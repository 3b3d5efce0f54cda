# GPU: the driver's exact bench command, then a 2-rank rehearsal of the
# multi-GPU flow on the one GPU (ranks share the device; each rank runs its
# 2 peer pipelines), then the round profile with the solo-window traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_r05ah.log 2>&1 || { tail -20 gpurun_out/bench_driver_r05ah.log; exit 1; }
tail -1 gpurun_out/bench_driver_r05ah.log | cut -c1-400
ORION_BENCH_REHEARSE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rehearse2_r05ah.log 2>&1 || { tail -30 gpurun_out/rehearse2_r05ah.log; exit 1; }
grep '^{' gpurun_out/rehearse2_r05ah.log | tail -1 | cut -c1-400
bash tools/gpu_prof.sh r05ah
