#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=gpurun_out/r05e
timeout -k 10 120 python -u tools/spd_timing.py > ${T}_spd_timing.log 2>&1; rc=$?; [ $rc -ne 0 ] && { cat ${T}_spd_timing.log; exit $rc; }
ADMMQ_LIB=$PWD/tools/tracelib/libadmmq.so timeout -k 10 120 python -u tools/spd_timing.py >> ${T}_spd_timing.log 2>&1; rc=$?
grep -v amdgpu.ids ${T}_spd_timing.log | tail -3; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_epc.py -x -q -rf -s --timeout 300 --timeout-method thread > ${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "parafac-epc|passed|failed|Error" ${T}_pytest.log | tail -8
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u tools/epc_profile.py > ${T}_epc_profile.log 2>&1; rc=$?; grep -v amdgpu.ids ${T}_epc_profile.log
exit $rc
