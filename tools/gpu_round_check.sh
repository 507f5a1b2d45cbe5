#!/bin/bash
# A round-end check on one GPU box: the whole GPU suite, smoke, the default bench
# line, then the kernel-trace stats of the default bench command (outputs gpurun_out/TAG_*).
# Usage: tools/gpu_round_check.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=gpurun_out/${1:-r05f}
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf -s --timeout 300 --timeout-method thread > ${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "C2 |C3 |parafac-epc|passed|failed|Error" ${T}_pytest.log | tail -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > ${T}_smoke.log 2>&1 || { cat ${T}_smoke.log; exit 5; }
tail -2 ${T}_smoke.log
timeout -k 10 300 python -u bench.py > ${T}_bench.json 2> ${T}_bench.err || { tail ${T}_bench.err; exit 6; }
tail -c 1200 ${T}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${T}_ktrace -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > ${T}_ktrace.log 2>&1 || { tail ${T}_ktrace.log; exit 7; }
echo ktrace done
