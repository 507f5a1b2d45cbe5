#!/bin/bash
# Round-3 session V: stage-1 units sized to fill the resident round evenly (A/B on C3 with
# ADMMQ_EVEN_UNITS=0, search phase timeline, parity tests); (f)3 low-rank timing with the
# Krylov projection checked against the exact truncation on the loop's own iterates;
# emulated 8-GPU layer shards of C3 / C4 on one GPU; C4 / C5 bench lines.
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "v_tests|600|python -u -m pytest -x -q -rf --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_parity.py" \
  "v_r18_even|300|python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline" \
  "v_r18_old|300|ADMMQ_EVEN_UNITS=0 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline" \
  "v_hist0|120|ADMMQ_LIB=$T python -u tools/hist_timeline.py --mode 0 --iters 6" \
  "v_lowrank|400|python -u tools/lowrank_bench.py" \
  "v_emu18|300|python -u bench.py --emulate-world 8 --steps 1 --warmup 1" \
  "v_emu50|300|python -u bench.py --model resnet50 --emulate-world 8 --steps 1 --warmup 1" \
  "v_r50|300|python -u bench.py --model resnet50 --steps 2 --warmup 1 --no-cpu-baseline" \
  "v_llama|400|python -u bench.py --model llama7b --steps 1 --warmup 1 --no-cpu-baseline"
