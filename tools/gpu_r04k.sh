#!/bin/bash
# Round-4 session K: panel kernels with end-anchored counters, the search's block selection
# restored; C3 bench + timelines, finalize-form A/B, low-rank bench and profile.
cd "$(dirname "$0")/.." || exit 1
V=$PWD/tools
bash tools/gpu_run.sh \
  "k_panel|240|python -u -m pytest tests/test_gpu_panel.py tests/test_gpu_lowrank.py -x -v --timeout 120 --timeout-method thread" \
  "k_bench|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "k_ns|200|ADMMQ_LIB=$V/varlib_ns/libadmmq.so python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "k_cur|200|ADMMQ_LIB=$V/varlib_cur/libadmmq.so python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "k_ht0|120|ADMMQ_LIB=$V/tracelib/libadmmq.so python -u tools/hist_timeline.py --mode 0 --iters 6" \
  "k_ht1|120|ADMMQ_LIB=$V/tracelib/libadmmq.so python -u tools/hist_timeline.py --shapes 512:1141 --iters 6" \
  "k_lrb|200|python -u tools/lowrank_bench.py --outer 6 --check 0,1 --svd-sample 0" \
  "k_lrprof|200|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k_lr -o lr -- python3 tools/lowrank_bench.py --outer 6 --check 0 --svd-sample 0" \
  "k_clean|60|find gpurun_out/k_lr -name '*kernel_trace*' -delete; find gpurun_out/k_lr -name '*.db' -delete; du -sh gpurun_out"
