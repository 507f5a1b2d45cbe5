#!/bin/bash
# Round-3 final evidence: the search setup with tie groups resolved in the threshold phase
# (stage-1 parity first), full GPU suite, smoke, C3 bench line with the CPU baseline,
# search phase timeline, rocprofv3 kernel-trace stats + PMC passes of the C3 bench.
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "f1_stage1|300|python -u -m pytest -x -q -rf --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k 'sse or stage1 or kat or exhaustive or f7 or small or fused'" || exit $?
grep -q " passed" gpurun_out/f1_stage1.log && ! grep -q "failed" gpurun_out/f1_stage1.log || { echo "stage-1 tests failed: stopping"; exit 1; }
bash tools/gpu_run.sh \
  "f1_suite|800|python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread" \
  "f1_smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "f1_r18|400|python -u bench.py" \
  "f1_hist0|120|ADMMQ_LIB=$T python -u tools/hist_timeline.py --mode 0 --iters 6" \
  "f1_prof|900|bash tools/profile.sh r03z resnet18"
