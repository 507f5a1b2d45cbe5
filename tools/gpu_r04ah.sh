#!/bin/bash
# Round-4 session AH (final tree after the SPD change): smoke, default bench line, C4 / C5.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "ah_smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "ah_bench|400|python -u bench.py" \
  "ah_c4|200|python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline" \
  "ah_c5|300|python -u bench.py --model llama7b --steps 2 --warmup 1 --no-cpu-baseline"
