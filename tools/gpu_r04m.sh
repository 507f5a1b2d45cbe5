#!/bin/bash
# Round-4 session M: three float4 groups per search thread at C4 (fused finalize), the
# LATE variant removed, Cholesky-QR Krylov: full GPU suite, C4 A/B, C3 bench.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "m_pytest|900|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "m_c4|300|python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline" \
  "m_c4_nv2|300|python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline --fin-nv3 0" \
  "m_c3|200|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline"
