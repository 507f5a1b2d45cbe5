#!/bin/bash
# Round-4 session AE: 256x128 tiles at C4 / C3 (wide-tile threshold forced to 0) vs default.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "ae_c4_def|200|python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline" \
  "ae_c4_wide|200|python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline --wide-min 0" \
  "ae_c3_wide|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --wide-min 0" \
  "ae_c4_w1500|200|python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline --wide-min 1000"
