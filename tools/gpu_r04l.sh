#!/bin/bash
# Round-4 session L: Cholesky-QR Krylov blocks, templated outer product, parallel lr_post
# tail: low-rank tests, the notebook-scale bench and its profile, the full (f)3 run.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "l_panel|240|python -u -m pytest tests/test_gpu_panel.py tests/test_gpu_lowrank.py -x -v --timeout 120 --timeout-method thread" \
  "l_lrb|200|python -u tools/lowrank_bench.py --outer 6 --check 0,1 --svd-sample 0" \
  "l_lrprof|200|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/l_lr -o lr -- python3 tools/lowrank_bench.py --outer 6 --check -5 --svd-sample 0" \
  "l_clean|60|find gpurun_out/l_lr -name '*kernel_trace*' -delete; find gpurun_out/l_lr -name '*.db' -delete; du -sh gpurun_out" \
  "l_f3|400|python -u tools/lowrank_bench.py --svd-sample 2"
