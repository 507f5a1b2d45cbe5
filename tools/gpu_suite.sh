#!/bin/bash
# One GPU box session: the GPU test suite (or the given pytest selection), then - only if
# it ended without a fault, abort or timeout - a default bench line. Outputs under
# gpurun_out/<tag>_*. Usage: tools/gpu_suite.sh TAG [pytest-args...]
cd "$(dirname "$0")/.." || exit 1
tag=${1:-run}; shift
mkdir -p gpurun_out
sel=("$@"); [ ${#sel[@]} -eq 0 ] && sel=(tests -m gpu)
timeout -k 10 1100 python -u -m pytest "${sel[@]}" -x -q -rf --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/${tag}_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
brc=$?
echo "bench rc=$brc"; tail -c 1500 gpurun_out/${tag}_bench.json
exit $brc
