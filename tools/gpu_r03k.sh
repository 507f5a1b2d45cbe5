#!/bin/bash
# Round-3 session K: full GPU suite, smoke, multi-GPU readiness (--emulate-world 8 for C4 and
# C3: every rank's LPT shard timed on this GPU), (f)3 low-rank timing.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
  > gpurun_out/k_tests.log 2>&1; rc=$?; tail -2 gpurun_out/k_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/k_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --model resnet50 --emulate-world 8 --steps 1 --warmup 1 > gpurun_out/k_emu_r50.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --model resnet18 --emulate-world 8 --steps 1 --warmup 1 > gpurun_out/k_emu_r18.log 2>&1 || exit $?
timeout -k 10 900 python -u tools/lowrank_bench.py > gpurun_out/k_lowrank.log 2>&1 || exit $?
echo done
