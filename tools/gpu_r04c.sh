#!/bin/bash
# Round-4 session C: K-split phase trace of a lone layer4 factor; search timelines (lone
# layer, C3 mode 0); C3 A/B of the balance pieces and the 2-deep staging ring (4 tiles/CU);
# emulated shards with costs (shard-model fit); channel / op / F10 / K-split tests.
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "c_pytest|500|python -u -m pytest tests/test_gpu_parity.py tests/test_torch_ops.py tests/test_gpu_lowrank.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread -k 'channel or ops or repair or f10 or krylov or ksplit or staging or c3_batched or thin or legacy'" \
  "c_tl1|120|ADMMQ_LIB=$T python -u tools/gemm_timeline.py --shapes 512:1141 --iters 6" \
  "c_ht1|120|ADMMQ_LIB=$T python -u tools/hist_timeline.py --shapes 512:1141 --iters 6" \
  "c_ht0|120|ADMMQ_LIB=$T python -u tools/hist_timeline.py --mode 0 --iters 6" \
  "c_b11|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --ksplit-bal 1:1" \
  "c_b00|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --ksplit-bal 0:1" \
  "c_bs2|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --ksplit-bal 1:1 --gemm-stage 2" \
  "c_bs2n|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --ksplit-bal 0:1 --gemm-stage 2" \
  "c_emu18|300|python -u bench.py --emulate-world 8 --steps 2 --warmup 1" \
  "c_emu50|400|python -u bench.py --emulate-world 8 --model resnet50 --steps 2 --warmup 1"
