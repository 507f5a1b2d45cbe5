#!/bin/bash
# Round-3 session F2: GEMM / search timed by events their dispatches record
# (hipExtLaunchKernelGGL) - bench lines C3 / C4 / C5 next to a rocprofv3 kernel trace of C3;
# the torch-ops / C-ABI tests that go through the changed launchers.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "f2_tests|600|python -u -m pytest -x -q -rf --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_torch_ops.py -k 'c3 or wide or ops'" \
  "f2_r18|400|python -u bench.py" \
  "f2_r50|300|python -u bench.py --model resnet50 --steps 2 --warmup 1 --no-cpu-baseline" \
  "f2_llama|400|python -u bench.py --model llama7b --steps 1 --warmup 1 --no-cpu-baseline" \
  "f2_ktrace|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f2/ktrace -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
