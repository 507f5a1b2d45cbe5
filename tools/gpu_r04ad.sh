#!/bin/bash
# Round-4 session AD (final tree): full GPU suite, smoke, default bench line, C4 / C5 lines.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "ad_gpu|900|python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread" \
  "ad_smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "ad_bench|400|python -u bench.py" \
  "ad_c4|200|python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline" \
  "ad_c5|300|python -u bench.py --model llama7b --steps 2 --warmup 1 --no-cpu-baseline"
