#!/bin/bash
# The EPC step's phase trace (TRACE library), the EPC tests and the EPC profile.
# Usage: tools/gpu_epc.sh TAG [trace]   (trace: the phase trace only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=gpurun_out/${1:-r05i}
ADMMQ_LIB=$PWD/tools/tracelib/libadmmq.so timeout -k 10 120 python -u tools/spd_timing.py > ${T}_spd_timing.log 2>&1; rc=$?
[ "$2" = trace ] && { grep -v amdgpu.ids ${T}_spd_timing.log | tail -6; exit $rc; }
grep -v amdgpu.ids ${T}_spd_timing.log | tail -4; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_epc.py -x -q -rf -s --timeout 200 --timeout-method thread > ${T}_pytest_epc.log 2>&1
rc=$?; echo "pytest epc rc=$rc"; grep -E "parafac-epc|passed|failed|Error|assert" ${T}_pytest_epc.log | tail -12
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u tools/epc_profile.py > ${T}_epc_profile.log 2>&1; rc2=$?; grep -v amdgpu.ids ${T}_epc_profile.log
exit $((rc + rc2))
