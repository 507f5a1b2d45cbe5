#!/bin/bash
# Round-3 session T: fp32 64x64 GEMM staging forms (ADMMQ_GEMM_F32_STAGE 0..3, same bits):
# C3 fp32 parity tests on the new default, per-workgroup timelines of each form at mode 0,
# and the C3 bench line.
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "t_tests|400|python -u -m pytest -x -q -rf --timeout 200 --timeout-method thread tests/test_gpu_configs.py -k 'c3 or c4 or wide'" \
  "t_tl0|120|ADMMQ_GEMM_F32_STAGE=0 ADMMQ_LIB=$T python -u tools/gemm_timeline.py --mode 0 --iters 6" \
  "t_tl1|120|ADMMQ_GEMM_F32_STAGE=1 ADMMQ_LIB=$T python -u tools/gemm_timeline.py --mode 0 --iters 6" \
  "t_tl2|120|ADMMQ_GEMM_F32_STAGE=2 ADMMQ_LIB=$T python -u tools/gemm_timeline.py --mode 0 --iters 6" \
  "t_tl3|120|ADMMQ_GEMM_F32_STAGE=3 ADMMQ_LIB=$T python -u tools/gemm_timeline.py --mode 0 --iters 6" \
  "t_r18|300|python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
