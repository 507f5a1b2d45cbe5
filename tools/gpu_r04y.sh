#!/bin/bash
# Round-4 session Y: next-unit prefetch in the multi-unit (non-fused) search - full GPU
# suite, C5 / C3 benches.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "y_gpu|900|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "y_c5|300|python -u bench.py --model llama7b --steps 2 --warmup 1 --no-cpu-baseline" \
  "y_c3|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline"
