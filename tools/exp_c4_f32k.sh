#!/bin/bash
# A/B: C4 (resnet50) solve kernel forms (bench.py --f32-kernel: -1 default, 1 persistent
# per-workgroup tile lists, 2 per-problem tile rows), interleaved twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
tag=${1:-c4k}
for rep in 1 2; do
  for k in -1 1 2; do
    timeout -k 10 300 python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline --f32-kernel $k \
      > gpurun_out/${tag}_k${k}_r$rep.json 2> gpurun_out/${tag}_k${k}_r$rep.err || exit 1
  done
done
