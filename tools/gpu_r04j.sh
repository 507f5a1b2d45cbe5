#!/bin/bash
# Round-4 session J: panel kernel tests + low-rank tests, search A/B against HEAD (bench and
# C3 mode-0 timelines from both trace builds), low-rank loop bench and profile.
cd "$(dirname "$0")/.." || exit 1
V=$PWD/tools
bash tools/gpu_run.sh \
  "j_panel|240|python -u -m pytest tests/test_gpu_panel.py tests/test_gpu_lowrank.py -x -v --timeout 120 --timeout-method thread" \
  "j_head|200|ADMMQ_LIB=$V/varlib_head/libadmmq.so python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "j_cur|200|ADMMQ_LIB=$V/varlib_cur/libadmmq.so python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "j_ht_head|120|ADMMQ_LIB=$V/varlib_headtr/libadmmq.so python -u tools/hist_timeline.py --mode 0 --iters 6" \
  "j_ht_cur|120|ADMMQ_LIB=$V/tracelib/libadmmq.so python -u tools/hist_timeline.py --mode 0 --iters 6" \
  "j_lrb|300|python -u tools/lowrank_bench.py --outer 6 --check 0,1 --svd-sample 0" \
  "j_lrprof|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/j_lr -o lr -- python3 tools/lowrank_bench.py --outer 6 --check 0 --svd-sample 0" \
  "j_clean|60|find gpurun_out/j_lr -name '*kernel_trace*' -delete; find gpurun_out/j_lr -name '*.db' -delete; du -sh gpurun_out"
