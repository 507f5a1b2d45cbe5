#!/bin/bash
# Round-3 session A: fp32-solve bench lines for C3 / C4 / C5 (the reference's arithmetic),
# then a kernel trace of the C3 fp32 form.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --solve fp32 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/a_r18_fp32.log 2>&1 || exit $?
tail -c 400 gpurun_out/a_r18_fp32.log
timeout -k 10 300 python -u bench.py --solve fp32 --model resnet50 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/a_r50_fp32.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --solve fp32 --model llama7b --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/a_llama_fp32.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/a_ktrace -o run -- \
  python3 bench.py --solve fp32 --steps 1 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/a_ktrace.log 2>&1 || exit $?
echo done
