# r04r: ResNet-20 N=2^16 and LoLA batch 1 over the latency-kernel threshold
# (ORION_NTT2S_BELOW) and the INTT-fusion redundancy limit (ORION_NTT_IFUSE_MAXR)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 128:8 256:8 128:32 256:32; do
  b=${v%:*}; r=${v#*:}
  ORION_NTT2S_BELOW=$b ORION_NTT_IFUSE_MAXR=$r WORKLOAD=resnet20_n16 BATCH=1 timeout -k 10 300 python -u tools/resnet_bench.py > gpurun_out/r04r_resnet_${b}_$r.log 2>&1 || { tail -20 gpurun_out/r04r_resnet_${b}_$r.log; exit 1; }
  echo "BELOW=$b MAXR=$r resnet: $(grep workload gpurun_out/r04r_resnet_${b}_$r.log | tail -1 | cut -c90-160)"
done
for v in 8 32; do
  ORION_NTT_IFUSE_MAXR=$v timeout -k 10 200 python bench.py --batch 1 --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/r04r_b1_$v.log 2>&1 || { tail -20 gpurun_out/r04r_b1_$v.log; exit 1; }
  echo "MAXR=$v batch1: $(tail -1 gpurun_out/r04r_b1_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/image")')"
done
