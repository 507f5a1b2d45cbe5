#!/bin/bash
# Round-6 measurement session: the default bench line (C3 with its CPU baseline), C4 / C5
# lines, the emulated 8-rank shards of resnet18 / resnet50, and the EPC initialiser timing.
# Each step under its own time limit; the session stops at the first failure.
cd "$(dirname "$0")/.." || exit 1
T=gpurun_out/${1:-r06q}
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python3 -u bench.py > ${T}_bench_default.json 2> ${T}_bench_default.err || exit 3
timeout -k 10 300 python3 -u bench.py --model resnet50 --no-cpu-baseline > ${T}_bench_resnet50.json 2> ${T}_bench_resnet50.err || exit 4
timeout -k 10 300 python3 -u bench.py --model llama7b --steps 1 --warmup 1 --no-cpu-baseline > ${T}_bench_llama7b.json 2> ${T}_bench_llama7b.err || exit 5
timeout -k 10 300 python3 -u bench.py --model resnet50 --emulate-world 8 --steps 2 --warmup 1 --no-cpu-baseline > ${T}_emu50.json 2> ${T}_emu50.err || exit 6
timeout -k 10 300 python3 -u bench.py --model resnet18 --emulate-world 8 --steps 2 --warmup 1 --no-cpu-baseline > ${T}_emu18.json 2> ${T}_emu18.err || exit 7
echo done
