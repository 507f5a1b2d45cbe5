#!/bin/bash
# Round-4 session P: full GPU suite (layer4 long horizon, Gram sum), search timelines with
# the selection latency (min of ticket->selection), low-rank runs, C3 bench.
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "p_pytest|900|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rA -k 'layer4_long or panel or lowrank or parity or configs'" \
  "p_ht0|120|ADMMQ_LIB=$T python -u tools/hist_timeline.py --mode 0 --iters 6" \
  "p_ht1|120|ADMMQ_LIB=$T python -u tools/hist_timeline.py --shapes 512:1141 --iters 6" \
  "p_lrb|200|python -u tools/lowrank_bench.py --outer 6 --check 0,1 --svd-sample 0" \
  "p_f3|400|python -u tools/lowrank_bench.py --svd-sample 2" \
  "p_c3|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline"
