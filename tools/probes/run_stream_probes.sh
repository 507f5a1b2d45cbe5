#!/usr/bin/env bash
# GEMM delivery / K-loop decomposition probes (see DESIGN.md "GEMM: what bounds it").
# Build here: hipcc -O3 --offload-arch=gfx950 tools/probes/stream_probe.hip -o tools/probes/stream_probe
# Run on the GPU box: bash tools/probes/run_stream_probes.sh > gpurun_out/stream_probes.log
set -e
P=tools/probes/stream_probe
run() { timeout -k 5 30 $P "$@"; }
# streaming only: one workgroup, all CUs private (miss traffic), all CUs shared (L2 hits)
run 0 1 1024 3 0; run 1 1 1024 3 0
run 0 256 256 5 0; run 1 256 256 5 0
run 0 256 256 5 1; run 1 256 256 5 1
# the GEMM's row pattern and its K-loop: {loads}, {+fragment reads}, {+MFMA}, {both}
for m in 2 3 4 5 6; do run $m 1 576 9 0; done
for m in 3 4 5 6; do run $m 144 576 9 1; done
# K-loop at 1/2/3 workgroups per CU, miss traffic vs L2 hits
run 6 256 576 9 0; run 6 512 576 9 0; run 6 768 576 9 0; run 6 768 576 9 1
