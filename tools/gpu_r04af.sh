#!/bin/bash
# Round-4 session AF: SPD-inverse kernel probe (C3 shape, 16 x R = 1141), with the
# LDS-broadcast chol32 variant.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh "af_spd|120|./tools/spd_probe.bin"
