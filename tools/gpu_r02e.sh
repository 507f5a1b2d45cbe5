#!/bin/bash
# Round-2 session D (part 2): the bench lines of C3 (default config, with the CPU
# baseline), C4 and C5 on the committed tree, reading profiles/r02_<model>_traffic.json.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r18.log 2>&1 || exit $?
tail -c 300 gpurun_out/bench_r18.log
timeout -k 10 500 python -u bench.py --model resnet50 --steps 3 --warmup 1 > gpurun_out/bench_r50.log 2>&1 || exit $?
tail -c 300 gpurun_out/bench_r50.log
timeout -k 10 500 python -u bench.py --model llama7b --steps 2 --warmup 1 > gpurun_out/bench_llama.log 2>&1 || exit $?
tail -c 300 gpurun_out/bench_llama.log
