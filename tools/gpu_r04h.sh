#!/bin/bash
# Round-4 session H: A/B of the fused finalize forms against HEAD's library at C3 (search
# launch average from the bench line), lone search timeline, low-rank loop profile.
cd "$(dirname "$0")/.." || exit 1
V=$PWD/tools
bash tools/gpu_run.sh \
  "h_head|200|ADMMQ_LIB=$V/varlib_head/libadmmq.so python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "h_cur|200|ADMMQ_LIB=$V/varlib_cur/libadmmq.so python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "h_ns|200|ADMMQ_LIB=$V/varlib_ns/libadmmq.so python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "h_head2|200|ADMMQ_LIB=$V/varlib_head/libadmmq.so python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "h_ops|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "h_lrprof|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/h_lr -o lr -- python3 tools/lowrank_bench.py --outer 6 --check 0 --svd-sample 0" \
  "h_clean|60|find gpurun_out/h_lr -name '*kernel_trace*' -delete; find gpurun_out/h_lr -name '*.db' -delete; du -sh gpurun_out"
