#!/bin/bash
# Round-4 session AA: search buckets zeroed while the stop flag / max|x| loads are in
# flight - search/config tests, C3 / C4 benches, lone shard, search timelines.
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "aa_tests|600|python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_reference.py -x -q --timeout 120 --timeout-method thread" \
  "aa_c3|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "aa_c4|200|python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline" \
  "aa_emu|200|python -u bench.py --emulate-world 8 --model resnet50 --emulate-only 0,3 --steps 2 --warmup 1" \
  "aa_ht0|120|ADMMQ_LIB=$T python -u tools/hist_timeline.py --mode 0 --iters 6" \
  "aa_ht1|120|ADMMQ_LIB=$T python -u tools/hist_timeline.py --shapes 512:1141 --iters 6"
