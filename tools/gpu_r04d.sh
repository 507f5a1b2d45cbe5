#!/bin/bash
# Round-4 session D: pinned-staging uploads (host planning off the critical path), balance
# A/B, thin-loop phases with predicated stage-1 atomics, K-split / search timelines.
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "d_b11|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --ksplit-bal 1:1" \
  "d_b00|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --ksplit-bal 0:1" \
  "d_r50|240|python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline" \
  "d_thin|200|ADMMQ_LIB=$T python -u tools/thin_loop_timeline.py" \
  "d_tl1|120|ADMMQ_LIB=$T python -u tools/gemm_timeline.py --shapes 512:1141 --iters 6" \
  "d_ht1|120|ADMMQ_LIB=$T python -u tools/hist_timeline.py --shapes 512:1141 --iters 6" \
  "d_ht0|120|ADMMQ_LIB=$T python -u tools/hist_timeline.py --mode 0 --iters 6" \
  "d_pytest|500|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k 'thin or legacy or batched or small or stage1 or fused'" \
  "d_emu50|400|python -u bench.py --emulate-world 8 --model resnet50 --steps 2 --warmup 1"
