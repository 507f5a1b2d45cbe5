#!/bin/bash
# Round-4 session I: the panel kernels (new) and the low-rank tests on them, the fused
# finalize A/B against HEAD's library at C3, low-rank loop profile.
cd "$(dirname "$0")/.." || exit 1
V=$PWD/tools
bash tools/gpu_run.sh \
  "i_panel|240|python -u -m pytest tests/test_gpu_panel.py tests/test_gpu_lowrank.py -x -v --timeout 120 --timeout-method thread" \
  "i_head|200|ADMMQ_LIB=$V/varlib_head/libadmmq.so python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "i_cur|200|ADMMQ_LIB=$V/varlib_cur/libadmmq.so python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "i_ns|200|ADMMQ_LIB=$V/varlib_ns/libadmmq.so python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "i_head2|200|ADMMQ_LIB=$V/varlib_head/libadmmq.so python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "i_lrb|300|python -u tools/lowrank_bench.py --outer 6 --check 0,1 --svd-sample 0" \
  "i_lrprof|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/i_lr -o lr -- python3 tools/lowrank_bench.py --outer 6 --check 0 --svd-sample 0" \
  "i_clean|60|find gpurun_out/i_lr -name '*kernel_trace*' -delete; find gpurun_out/i_lr -name '*.db' -delete; du -sh gpurun_out"
