#!/bin/bash
# Round-4 session F: low-rank (f)3 kernel profile (stats only kept), emulated shards after
# the stage-1 unit revert, C3 bench.
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "f_lrprof|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f_lr -o lr -- python3 tools/lowrank_bench.py --outer 6 --check 0 --svd-sample 1" \
  "f_clean|60|find gpurun_out/f_lr -name '*kernel_trace*' -delete; find gpurun_out/f_lr -name '*.db' -delete; du -sh gpurun_out" \
  "f_emu50|400|python -u bench.py --emulate-world 8 --model resnet50 --steps 2 --warmup 1" \
  "f_ht1|120|ADMMQ_LIB=$T python -u tools/hist_timeline.py --shapes 512:1141 --iters 6"
