#!/bin/bash
# Round-3 session U: scalar-offset fp32 staging (k_gemm_f32b<3, false>, default) with the
# grid padded to whole rounds (every CU may take 3 tiles): GPU configs + parity tests,
# GEMM timelines of modes 0 and 1, C3 bench line.
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "u_tests|600|python -u -m pytest -x -q -rf --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_parity.py" \
  "u_tl0|120|ADMMQ_LIB=$T python -u tools/gemm_timeline.py --mode 0 --iters 6" \
  "u_tl1|120|ADMMQ_LIB=$T python -u tools/gemm_timeline.py --mode 1 --iters 6" \
  "u_r18|300|python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
