#!/bin/bash
# Round-3 final evidence (F3): GEMM / search timed by events their own dispatches record
# (hipExtLaunchKernelGGL); full GPU suite, smoke, C3 bench line with the CPU baseline,
# C4 / C5 bench lines, rocprofv3 kernel-trace stats + PMC passes of C3, search timeline.
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "f3_suite|800|python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread" \
  "f3_smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "f3_r18|400|python -u bench.py" \
  "f3_r50|300|python -u bench.py --model resnet50 --steps 2 --warmup 1 --no-cpu-baseline" \
  "f3_llama|400|python -u bench.py --model llama7b --steps 1 --warmup 1 --no-cpu-baseline" \
  "f3_prof|900|bash tools/profile.sh r03f resnet18" \
  "f3_hist0|120|ADMMQ_LIB=$T python -u tools/hist_timeline.py --mode 0 --iters 6"
