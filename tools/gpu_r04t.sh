#!/bin/bash
# Round-4 session T: C5 (Llama-7B layer) rocprofv3 evidence on the round-4 tree.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh "t_prof_llama|1000|bash tools/profile.sh r04 llama7b"
