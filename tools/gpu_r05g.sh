#!/bin/bash
# Round 5 session g: the tridiagonal EPC step (tests + profile), then the horizon tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=gpurun_out/r05g
timeout -k 10 300 python -u -m pytest tests/test_gpu_epc.py -x -q -rf -s --timeout 200 --timeout-method thread > ${T}_pytest_epc.log 2>&1
rc=$?; echo "pytest epc rc=$rc"; grep -E "parafac-epc|passed|failed|Error|assert" ${T}_pytest_epc.log | tail -12
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u tools/epc_profile.py > ${T}_epc_profile.log 2>&1; rc2=$?; grep -v amdgpu.ids ${T}_epc_profile.log
[ $rc2 -ne 0 ] && exit $rc2
timeout -k 10 600 python -u -m pytest tests/test_gpu_horizon.py -x -q -rf -s --timeout 400 --timeout-method thread > ${T}_pytest_horizon.log 2>&1
rc3=$?; echo "pytest horizon rc=$rc3"; grep -E "C2 |C3 |passed|failed|Error" ${T}_pytest_horizon.log | tail -12
exit $((rc + rc3))
