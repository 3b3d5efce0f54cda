# GPU: parity suite with the giant-split kernels (auto at batch <= 2), then a
# batch-1 / B=64 A/B of the two split switches, then the batch-1 kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05ai_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r05ai_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r05ai_gpu_tests.log
for r in 1 2; do
  for v in off auto bsgs_only giant_only giant2; do
    case $v in
      off) E="ORION_LT_GSPLIT=1 ORION_LT_GIANT_SPLIT=1";;
      auto) E="ORION_LT_GSPLIT=0";;
      bsgs_only) E="ORION_LT_GIANT_SPLIT=1";;
      giant_only) E="ORION_LT_GSPLIT=1";;
      giant2) E="ORION_LT_GIANT_SPLIT=2";;
    esac
    o=gpurun_out/r05ai_${v}_$r.log
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $o 2>&1 || { tail -20 $o; exit 1; }
    echo "$v $r: $(tail -1 $o | python -c 'import json,sys; d=json.loads(sys.stdin.read()); b=d["batch1"]; print("batch1 graph", b["ms_per_image"], "stream", b["stream_ms_per_image"], "ms; B=64", d["value"], "img/s lt", d["kernel_ms_per_step"]["lt_bsgs"], d["kernel_ms_per_step"]["lt_giant"])')"
  done
done
bash tools/gpu_b1_prof.sh r05ai > gpurun_out/prof_b1_r05ai_stats.txt 2>&1 || { tail -20 gpurun_out/prof_b1_r05ai_stats.txt; exit 1; }
f=$(find gpurun_out/prof_b1_r05ai -name "b1_kernel_trace.csv" | head -1)
python tools/b1_trace_summ.py "$f" 20 > gpurun_out/prof_b1_r05ai_trace_summary.txt && cat gpurun_out/prof_b1_r05ai_trace_summary.txt
