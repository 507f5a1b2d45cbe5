#!/bin/bash
# Round-4 session G: spill-free fused search (one unit per block), quantize statistics
# without same-address atomics, float4 low-rank streams: full GPU suite, C3 bench, lone
# search timeline, low-rank loop profile (no exact-SVD sample).
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "g_pytest|900|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "g_bench|300|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "g_ht1|120|ADMMQ_LIB=$T python -u tools/hist_timeline.py --shapes 512:1141 --iters 6" \
  "g_lrprof|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g_lr -o lr -- python3 tools/lowrank_bench.py --outer 6 --check 0 --svd-sample 0" \
  "g_clean|60|find gpurun_out/g_lr -name '*kernel_trace*' -delete; find gpurun_out/g_lr -name '*.db' -delete; du -sh gpurun_out"
