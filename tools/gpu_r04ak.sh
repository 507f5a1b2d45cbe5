#!/bin/bash
# Round-4 session AK (final tree): full GPU suite and smoke.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "ak_gpu|900|python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread" \
  "ak_smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
