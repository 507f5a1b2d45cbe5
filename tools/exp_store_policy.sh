#!/bin/bash
# A/B (diagnostics): store policy variants tools/ablib/ntV (built with EXTRA=-DADMMQ_SC1_STORES=V
# on top of the default nontemporal policy) on C3 and C4, interleaved twice; same bits.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
tag=${1:-sp}
for rep in 1 2; do
  for v in ${VARIANTS:-0 2 4 6 7}; do
    export ADMMQ_LIB=$PWD/tools/ablib/nt$v/libadmmq.so
    timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_c3_v${v}_r$rep.json 2> gpurun_out/${tag}_c3_v${v}_r$rep.err || exit 1
    timeout -k 10 200 python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_c4_v${v}_r$rep.json 2> gpurun_out/${tag}_c4_v${v}_r$rep.err || exit 1
  done
done
