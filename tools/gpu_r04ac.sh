#!/bin/bash
# Round-4 session AC (final tree): emulated 8-GPU shards of C3 and C4 for the shard-model
# refit, and the 4-rank emulation for the model's check at another world size.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "ac_emu18|300|python -u bench.py --emulate-world 8 --steps 2 --warmup 1" \
  "ac_emu50|300|python -u bench.py --emulate-world 8 --model resnet50 --steps 2 --warmup 1" \
  "ac_emu50w4|300|python -u bench.py --emulate-world 4 --model resnet50 --steps 2 --warmup 1"
