#!/bin/bash
# Round-4 session U: lone layer4 GEMM placement (parallel K-split pieces) and the effect of
# capping the pieces' workgroups per CU; emulated shards 0 (lone layer4) and 3 (7 layers).
cd "$(dirname "$0")/.." || exit 1
T=$PWD/tools/tracelib/libadmmq.so
bash tools/gpu_run.sh \
  "u_tl0|120|ADMMQ_LIB=$T python -u tools/gemm_timeline.py --shapes 512:1141 --iters 6" \
  "u_tl8k|120|ADMMQ_LIB=$T python -u tools/gemm_timeline.py --shapes 512:1141 --iters 6 --par-lds 8192" \
  "u_emu0|200|python -u bench.py --emulate-world 8 --model resnet50 --emulate-only 0,3 --steps 2 --warmup 1" \
  "u_emu8k|200|python -u bench.py --emulate-world 8 --model resnet50 --emulate-only 0,3 --steps 2 --warmup 1 --par-lds 8192"
