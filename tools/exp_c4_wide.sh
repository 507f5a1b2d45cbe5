#!/bin/bash
# A/B: C4 (resnet50) with the 256 x 128 wide tiles from 1000 / 1400 64x64 tiles per launch
# against the default threshold (kWideMinTiles); same bits.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
tag=${1:-c4w}
for wm in -1 1400 1000; do
  timeout -k 10 300 python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline --wide-min $wm \
    > gpurun_out/${tag}_wm$wm.json 2> gpurun_out/${tag}_wm$wm.err || exit 1
done
