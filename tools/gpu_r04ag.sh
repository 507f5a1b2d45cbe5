#!/bin/bash
# Round-4 session AG: trinv32 with each row's entries read before its FMA chains (same
# bits) - SPD probe, full GPU suite, C3 bench, lone-layer shard.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "ag_spd|120|./tools/spd_probe.bin" \
  "ag_gpu|900|python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread" \
  "ag_c3|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "ag_emu|200|python -u bench.py --emulate-world 8 --model resnet50 --emulate-only 0,3 --steps 2 --warmup 1"
