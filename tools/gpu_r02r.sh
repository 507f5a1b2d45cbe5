#!/bin/bash
# Round-2 session R: C5 search-units-per-block sweep (A/B of the planner's choice, 4 at C5).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for u in 0 2 6 8; do
  timeout -k 10 200 python -u bench.py --model llama7b --steps 1 --warmup 1 --no-cpu-baseline --search-units $u \
    > gpurun_out/bench_r_u$u.log 2>&1 || exit $?
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_r_u$u.log') if l.startswith('{')][-1]); print('units $u', round(d['value']), round(d['ms_per_step'],1), {k: round(v,1) for k,v in d['kernel_avg_us'].items()})"
done
