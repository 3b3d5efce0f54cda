# GPU: LoLA N=2^15 throughput / latency vs images per launch (bench.py --batch)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in 1 8 32 64 128 256; do
  timeout -k 10 300 python bench.py --batch $b --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sweep_b$b.txt 2>&1 || { tail -5 gpurun_out/sweep_b$b.txt; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep_b$b.txt').read().strip().splitlines()[-1]); print('B=$b', d['value'], 'img/s', d['ms_per_step'], 'ms/step', 'ntt_frac', d['roofline']['frac'])"
done
