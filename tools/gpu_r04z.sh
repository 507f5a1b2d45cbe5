#!/bin/bash
# Round-4 session Z (final-tree evidence): rocprofv3 kernel stats + PMC passes for C3 and
# C4, the default bench line (CPU baseline included), smoke.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "z_prof18|600|bash tools/profile.sh r04 resnet18" \
  "z_prof50|600|bash tools/profile.sh r04 resnet50" \
  "z_bench|400|python -u bench.py" \
  "z_smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
