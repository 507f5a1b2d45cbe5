#!/bin/bash
# Round-4 session AL (final tree): the default bench line with its CPU-baseline leg.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh "al_bench|400|python -u bench.py"
