#!/bin/bash
# Round-3 final evidence: full GPU suite, smoke, C3 bench line with the CPU baseline,
# rocprofv3 kernel-trace stats + PMC passes of the C3 bench (tools/profile.sh).
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "f1_suite|800|python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread" \
  "f1_smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "f1_r18|400|python -u bench.py" \
  "f1_prof|900|bash tools/profile.sh r03z resnet18"
