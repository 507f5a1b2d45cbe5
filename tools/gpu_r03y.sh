#!/bin/bash
# Round-3 session Y: C4 with the fused finalize on several units per block (capacity
# override 512 -> 2 units per block) against the separate finalize launch.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "y_r50_base|300|python -u bench.py --model resnet50 --steps 2 --warmup 1 --no-cpu-baseline" \
  "y_r50_fin512|300|ADMMQ_FIN_CAPACITY=512 python -u bench.py --model resnet50 --steps 2 --warmup 1 --no-cpu-baseline" \
  "y_r50_fin480|300|ADMMQ_FIN_CAPACITY=480 python -u bench.py --model resnet50 --steps 2 --warmup 1 --no-cpu-baseline"
