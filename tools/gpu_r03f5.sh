#!/bin/bash
# Round-3 session F5: k_gemm (wide 256x128, 32x64 and the split form's tiles) staged by
# scalar-offset buffer loads like k_gemm_f32b: GPU configs / parity / torch-ops suites,
# C5 / C3 bench lines.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "f5_tests|700|python -u -m pytest -x -q -rf --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_torch_ops.py" \
  "f5_llama|400|python -u bench.py --model llama7b --steps 1 --warmup 1 --no-cpu-baseline" \
  "f5_r18|300|python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline" \
  "f5_r18_split|300|python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --solve split"
