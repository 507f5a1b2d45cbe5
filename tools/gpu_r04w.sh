#!/bin/bash
# Round-4 session W: the single selected candidate carried in the fused finalize's ready
# word (no record stores / drain before it) - full GPU suite, C3 / C4 benches, lone-layer
# shard, search timelines.
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "w_gpu|900|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "w_c3|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "w_c4|200|python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline" \
  "w_emu|200|python -u bench.py --emulate-world 8 --model resnet50 --emulate-only 0,3 --steps 2 --warmup 1" \
  "w_ht0|120|ADMMQ_LIB=$T python -u tools/hist_timeline.py --mode 0 --iters 6" \
  "w_ht1|120|ADMMQ_LIB=$T python -u tools/hist_timeline.py --shapes 512:1141 --iters 6"
