#!/bin/bash
# Round 5 session h: workgroup barrier cost by size; EPC step phase trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=gpurun_out/r05h
for nt in 64 256 512 1024; do timeout -k 5 60 tools/probes/wg_barrier_probe $nt 2000 >> ${T}_wg_barrier.log 2>&1 || exit $?; done
cat ${T}_wg_barrier.log
ADMMQ_LIB=$PWD/tools/tracelib/libadmmq.so timeout -k 10 120 python -u tools/spd_timing.py > ${T}_spd_timing.log 2>&1; rc=$?
grep -v amdgpu.ids ${T}_spd_timing.log | tail -8; exit $rc
