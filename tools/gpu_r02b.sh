#!/bin/bash
# Round-2 GPU session B: C4 / C5 bench lines (with CPU baselines), the O1 end-to-end
# test, the (f)3 low-rank timing, then the C4 / C5 rocprof profiles.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_factorize_e2e.py -q -rf --timeout 150 --timeout-method thread \
  > gpurun_out/e2e.log 2>&1; rc=$?; tail -3 gpurun_out/e2e.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u bench.py --model resnet50 --steps 3 --warmup 1 > gpurun_out/bench_r50.log 2>&1 || exit $?
tail -c 400 gpurun_out/bench_r50.log
timeout -k 10 600 python -u bench.py --model llama7b --steps 2 --warmup 1 > gpurun_out/bench_llama.log 2>&1 || exit $?
tail -c 400 gpurun_out/bench_llama.log
timeout -k 10 600 python -u tools/lowrank_bench.py > gpurun_out/lowrank.log 2>&1 || exit $?
tail -c 800 gpurun_out/lowrank.log
timeout -k 10 500 bash tools/profile.sh r02 resnet50 || exit $?
timeout -k 10 500 bash tools/profile.sh r02 llama7b || exit $?
