#!/bin/bash
# Round-4 session E: cached tile plans + balance A/B, U prefetch in parallel K-split launches,
# even stage-1 units for small launches; full GPU suite; low-rank (f)3 kernel profile.
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "e_b11|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --ksplit-bal 1:1" \
  "e_b00|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --ksplit-bal 0:1" \
  "e_emu50|400|python -u bench.py --emulate-world 8 --model resnet50 --steps 2 --warmup 1" \
  "e_tl1|120|ADMMQ_LIB=$T python -u tools/gemm_timeline.py --shapes 512:1141 --iters 6" \
  "e_ht1|120|ADMMQ_LIB=$T python -u tools/hist_timeline.py --shapes 512:1141 --iters 6" \
  "e_thin|200|ADMMQ_LIB=$T python -u tools/thin_loop_timeline.py" \
  "e_suite|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "e_lrprof|300|rocprofv3 --kernel-trace --stats -d gpurun_out/e_lr -o lr -- python3 tools/lowrank_bench.py --outer 6 --check 0 --svd-sample 1"
