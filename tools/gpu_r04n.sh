#!/bin/bash
# Round-4 session N: fp64 Gram kernel tests, low-rank bench (6 outer + the notebook's 100),
# then the r04 rocprofv3 evidence for C3 (kernel-trace stats + separate PMC passes).
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "n_panel|240|python -u -m pytest tests/test_gpu_panel.py tests/test_gpu_lowrank.py -x -v --timeout 120 --timeout-method thread" \
  "n_lrb|200|python -u tools/lowrank_bench.py --outer 6 --check 0,1 --svd-sample 0" \
  "n_f3|400|python -u tools/lowrank_bench.py --svd-sample 2" \
  "n_prof18|900|bash tools/profile.sh r04 resnet18"
