#!/bin/bash
# Round 5 session d: EPC tests and profile (evaluation counts), C3 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=gpurun_out/r05d
timeout -k 10 600 python -u -m pytest tests/test_gpu_epc.py tests/test_gpu_configs.py -x -q -rf -s --timeout 300 \
  --timeout-method thread > ${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "parafac-epc|passed|failed|Error" ${T}_pytest.log | tail -8
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u tools/epc_profile.py > ${T}_epc_profile.log 2>&1; rc=$?; grep -v amdgpu.ids ${T}_epc_profile.log
exit $rc
