#!/usr/bin/env bash
# rocprofv3 evidence for profiles/: kernel-trace stats of the bench command, then
# separate PMC passes (FETCH_SIZE and WRITE_SIZE cannot share one pass on gfx950; SQ
# and TCC counters in passes of their own) on a shortened schedule (20 ADMM
# iterations) so counter replay stays quick.
# usage: tools/profile.sh <tag> [model] [extra bench args...]
set -u
tag="${1:-r02}"
model="${2:-resnet18}"
shift 2 2>/dev/null || shift $#
extra="$*"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/prof_${tag}_${model}
mkdir -p "$out"
short="--model $model --steps 1 --warmup 0 --max-iter-admm 21 --no-cpu-baseline --no-profile $extra"
run() {  # name seconds rocprof-args...
  local name=$1 secs=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$secs" rocprofv3 "$@" > "$out/$name.log" 2>&1
  local rc=$?
  tail -n 3 "$out/$name.log"
  if grep -qE "illegal memory access|Memory access fault|HSA_STATUS_ERROR" "$out/$name.log"; then echo "fault"; exit 3; fi
  if [ $rc -ne 0 ]; then echo "=== $name rc=$rc: stopping"; exit $rc; fi
}
run ktrace 600 --kernel-trace --stats --output-format csv -d "$out/ktrace" -o run -- \
    python3 bench.py --model "$model" --steps 2 --warmup 1 --no-cpu-baseline --no-profile $extra
run pmc_fetch 300 --pmc FETCH_SIZE --output-format csv -d "$out/pmc_fetch" -o run -- python3 bench.py $short
run pmc_write 300 --pmc WRITE_SIZE --output-format csv -d "$out/pmc_write" -o run -- python3 bench.py $short
run pmc_sq 300 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS \
    SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d "$out/pmc_sq" -o run -- python3 bench.py $short
run pmc_tcc 300 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$out/pmc_tcc" -o run -- python3 bench.py $short
echo "=== done"
