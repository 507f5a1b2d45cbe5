#!/bin/bash
# A/B (diagnostics): tools/ablib/{old,new}/libadmmq.so through ADMMQ_LIB on C5 and C3,
# interleaved twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
tag=${1:-on}
for rep in 1 2; do
  for v in old new; do
    export ADMMQ_LIB=$PWD/tools/ablib/$v/libadmmq.so
    timeout -k 10 300 python -u bench.py --model llama7b --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_c5_${v}_r$rep.json 2> gpurun_out/${tag}_c5_${v}_r$rep.err || exit 1
    timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_c3_${v}_r$rep.json 2> gpurun_out/${tag}_c3_${v}_r$rep.err || exit 1
  done
done
