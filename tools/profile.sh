#!/usr/bin/env bash
# rocprofv3 evidence for profiles/: kernel-trace stats of the bench command, then
# separate PMC passes (FETCH_SIZE and WRITE_SIZE cannot share one pass on gfx950)
# on a shortened schedule (20 ADMM iterations) so counter replay stays quick.
# usage: tools/profile.sh <tag>
set -u
tag="${1:-r01}"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/prof_${tag}
mkdir -p "$out"
short="--steps 1 --warmup 0 --max-iter-admm 21 --no-cpu-baseline --no-profile"
run() {  # name seconds rocprof-args...
  local name=$1 secs=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$secs" rocprofv3 "$@" > "$out/$name.log" 2>&1
  local rc=$?
  tail -n 5 "$out/$name.log"
  if grep -qE "illegal memory access|Memory access fault|HSA_STATUS_ERROR" "$out/$name.log"; then echo "fault"; exit 3; fi
  if [ $rc -ne 0 ]; then echo "=== $name rc=$rc: stopping"; exit $rc; fi
}
run ktrace 600 --kernel-trace --stats --output-format csv -d "$out/ktrace" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile
run pmc_fetch 600 --pmc FETCH_SIZE --output-format csv -d "$out/pmc_fetch" -o run -- python3 bench.py $short
run pmc_write 600 --pmc WRITE_SIZE --output-format csv -d "$out/pmc_write" -o run -- python3 bench.py $short
run pmc_sq 600 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS \
    --output-format csv -d "$out/pmc_sq" -o run -- python3 bench.py $short
echo "=== done"
find "$out" -name "*.csv" | head -50
