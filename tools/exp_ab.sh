#!/bin/bash
# A/B of an environment switch on the C3 bench (kernel averages per class). usage: exp_ab.sh VAR v1 v2 ...
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
var=$1; shift
for v in "$@"; do
  export $var=$v
  timeout -k 10 120 python bench.py --steps 2 --warmup 1 --max-iter-admm 201 --no-cpu-baseline --prof-every 4 \
    > gpurun_out/ab_${var}_$v.log 2>&1 || exit 1
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/ab_${var}_$v.log') if l.startswith('{')][-1]); print('$var=$v', {k: round(v,2) for k,v in d['kernel_avg_us'].items()}, round(d['ms_per_step'],2))"
done
