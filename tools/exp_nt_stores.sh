#!/bin/bash
# A/B (diagnostics): the C3 step with the solve / finalize outputs as nontemporal stores
# (tools/ablib/ntV built with EXTRA=-DADMMQ_NT_STORES=V: bit 0 H/U, bit 1 P, bit 2 H_T;
# same bits), every variant through ADMMQ_LIB, interleaved twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
tag=${1:-nt}
for rep in 1 2 3; do
  for v in ${VARIANTS:-0 3 4 7}; do
    ADMMQ_LIB=$PWD/tools/ablib/nt$v/libadmmq.so timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 \
      --no-cpu-baseline > gpurun_out/${tag}_nt${v}_r$rep.json 2> gpurun_out/${tag}_nt${v}_r$rep.err || exit 1
  done
done
