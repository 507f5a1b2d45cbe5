#!/bin/bash
# Round-3 rocprofv3 evidence for C4 and C5 on the final tree (kernel-trace stats + PMC passes).
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "f7_prof50|600|bash tools/profile.sh r03f resnet50" \
  "f7_profllama|800|bash tools/profile.sh r03f llama7b"
