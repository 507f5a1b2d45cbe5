#!/bin/bash
# Round-4 session B: K-split with serial / parallel execution forms; fault-repair paths.
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "b_pytest|500|python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_torch_ops.py tests/test_gpu_lowrank.py -x -v --timeout 300 --timeout-method thread -k 'ksplit or staging or wide or batched or c3_resnet18 or fault or repair or channel or krylov or ops'" \
  "b_bench|240|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "b_bench_r50|240|python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline" \
  "b_emu50|400|python -u bench.py --emulate-world 8 --model resnet50 --steps 2 --warmup 1" \
  "b_tl1|120|ADMMQ_LIB=$T python -u tools/gemm_timeline.py --shapes 512:1141 --iters 6"
