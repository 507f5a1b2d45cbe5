#!/usr/bin/env bash
# Kernel trace of a short bench run (100 ADMM iterations) into gpurun_out/<tag>.
# usage: tools/ktrace.sh <tag> [extra bench args]
set -u
tag="$1"; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag -o run -- \
  python3 bench.py --steps 1 --warmup 0 --max-iter-admm 101 --no-cpu-baseline --no-profile "$@" > gpurun_out/$tag.log 2>&1
