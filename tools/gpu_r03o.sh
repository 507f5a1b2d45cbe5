#!/bin/bash
# Round-3 session O: thin loop with the stop test behind the solve, candidate scales in LDS,
# every-wave barrier polling: parity, phase breakdown, C3 bench.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 120 --timeout-method thread \
  -k "thin or timeout or batched_equals_single or iteration_count" > gpurun_out/o_thin.log 2>&1
rc=$?; tail -2 gpurun_out/o_thin.log; [ $rc -eq 0 ] || exit $rc
ADMMQ_LIB=$PWD/tools/tracelib/libadmmq.so timeout -k 10 300 python -u tools/thin_loop_timeline.py \
  > gpurun_out/o_tl_r18.log 2>&1 || exit $?
tail -17 gpurun_out/o_tl_r18.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/o_r18.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/o_r50.log 2>&1 || exit $?
python3 -c "
import json
for f in ['gpurun_out/o_r18.log','gpurun_out/o_r50.log']:
    for l in open(f):
        if l.startswith('{'):
            d=json.loads(l); print(f, round(d['value']), round(d['ms_per_step'],1), {k: round(v,1) for k,v in d.get('kernel_ms_per_step',{}).items()})
"
echo done
