#!/bin/bash
# Round-4 session Q (final-tree evidence): full GPU suite, smoke, the default bench line
# (with its CPU baseline), C4 / C5 lines, search timelines, the (f)3 run.
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "q_pytest|900|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "q_smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "q_bench|400|python -u bench.py" \
  "q_r50|300|python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline" \
  "q_llama|400|python -u bench.py --model llama7b --steps 2 --warmup 1 --no-cpu-baseline" \
  "q_ht0|120|ADMMQ_LIB=$T python -u tools/hist_timeline.py --mode 0 --iters 6" \
  "q_ht1|120|ADMMQ_LIB=$T python -u tools/hist_timeline.py --shapes 512:1141 --iters 6" \
  "q_f3|400|python -u tools/lowrank_bench.py --svd-sample 2"
