#!/bin/bash
# Round-4 session X: thin-loop barrier 1 as tagged per-rank arrival words carrying max|X|
# (no counter, no second load) - thin-loop tests, C3 bench, phase breakdown, lone shard.
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "x_tests|400|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k 'thin or fault or repair or fused'" \
  "x_c3|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "x_tl|200|ADMMQ_LIB=$T python -u tools/thin_loop_timeline.py" \
  "x_emu|200|python -u bench.py --emulate-world 8 --model resnet50 --emulate-only 0,3 --steps 2 --warmup 1"
