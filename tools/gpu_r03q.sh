#!/bin/bash
# Round-3 session Q (re-entry): full GPU suite, smoke, C3/C4/C5 bench lines on HEAD.
cd "$(dirname "$0")/.." || exit 1
exec_steps=tools/gpu_run.sh
bash $exec_steps \
  "q_suite|700|python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread" \
  "q_smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "q_r18|300|python -u bench.py" \
  "q_r50|300|python -u bench.py --model resnet50 --steps 2 --warmup 1 --no-cpu-baseline" \
  "q_llama|400|python -u bench.py --model llama7b --steps 1 --warmup 1 --no-cpu-baseline"
