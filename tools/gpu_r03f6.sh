#!/bin/bash
# Round-3 final check on the committed tree: full GPU suite, smoke, C3 bench line with the
# CPU baseline, C4 bench line.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "f6_suite|800|python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread" \
  "f6_smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "f6_r18|400|python -u bench.py" \
  "f6_r50|300|python -u bench.py --model resnet50 --steps 2 --warmup 1 --no-cpu-baseline"
