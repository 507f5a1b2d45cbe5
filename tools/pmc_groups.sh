#!/usr/bin/env bash
# PMC passes, one counter group per rocprofv3 run (kernel-trace only), on a short bench.
# usage: tools/pmc_groups.sh <tag> "CNT_A CNT_B ..." ["CNT_C ..."] ...
set -u
tag="$1"; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p "$out"
short="--steps 1 --warmup 0 --max-iter-admm 21 --no-cpu-baseline --no-profile"
i=0
for grp in "$@"; do
  i=$((i+1))
  echo "=== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- python3 bench.py $short > "$out/p$i.log" 2>&1
  rc=$?
  if grep -qE "illegal memory access|Memory access fault|HSA_STATUS_ERROR" "$out/p$i.log"; then echo fault; exit 3; fi
  if [ $rc -ne 0 ]; then tail -5 "$out/p$i.log"; echo "rc=$rc"; exit $rc; fi
done
echo done
