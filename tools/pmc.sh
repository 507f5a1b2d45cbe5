#!/usr/bin/env bash
# PMC passes (one counter group per run, kernel-trace only) for the hot kernels.
# usage: tools/pmc.sh <tag>
set -u
tag="${1:-pmc}"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p "$out"
short="--steps 1 --warmup 0 --max-iter-admm 21 --no-cpu-baseline --no-profile"
i=0
for grp in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
  "TCC_HIT_sum TCC_MISS_sum" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LEVEL_WAVES SQ_INSTS_BRANCH SQ_INSTS_LDS_ATOMIC"; do
  i=$((i+1))
  echo "=== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- python3 bench.py $short > "$out/p$i.log" 2>&1
  rc=$?
  if grep -qE "illegal memory access|Memory access fault|HSA_STATUS_ERROR" "$out/p$i.log"; then echo fault; exit 3; fi
  if [ $rc -ne 0 ]; then tail -5 "$out/p$i.log"; echo "rc=$rc"; exit $rc; fi
done
echo done
