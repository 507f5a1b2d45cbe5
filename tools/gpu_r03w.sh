#!/bin/bash
# Round-3 session W: per-shard kernel averages of the emulated 8-GPU C3 run; thin-loop
# phase breakdown (C3 mode 2); single-layer GEMM timeline (layer4 conv, mode 0).
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "w_emu18|300|python -u bench.py --emulate-world 8 --steps 1 --warmup 1" \
  "w_thin|200|ADMMQ_LIB=$T python -u tools/thin_loop_timeline.py" \
  "w_tl1layer|120|ADMMQ_LIB=$T python -u tools/gemm_timeline.py --shapes 512:1141 --iters 6"
