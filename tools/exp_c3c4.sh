#!/bin/bash
# C3 and C4 bench lines, interleaved twice (store-policy checks)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
tag=${1:-c3c4}
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_c3_r$rep.json 2> gpurun_out/${tag}_c3_r$rep.err || exit 1
  timeout -k 10 300 python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_c4_r$rep.json 2> gpurun_out/${tag}_c4_r$rep.err || exit 1
done
