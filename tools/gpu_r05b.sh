#!/bin/bash
# Round 5 session b: GPU suite on the tree, then search-form A/B (per-level stage 1,
# one block per CU) on the lone layer4 factor and the emulated resnet50 shards.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=gpurun_out/r05b
sel=("$@"); [ ${#sel[@]} -eq 0 ] && sel=(tests -m gpu)
timeout -k 10 900 python -u -m pytest "${sel[@]}" -x -q -rf --timeout 300 --timeout-method thread > ${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 ${T}_pytest.log; [ $rc -ne 0 ] && exit $rc
for v in "0 0" "0 1" "2 0" "2 1"; do
  set -- $v
  echo "== timeline lone layer4 pl=$1 spread=$2" >> ${T}_timeline.log
  ADMMQ_LIB=$PWD/tools/tracelib/libadmmq.so timeout -k 10 120 python -u tools/hist_timeline.py --shapes 512:1141 \
    --iters 6 --pl $1 --spread $2 >> ${T}_timeline.log 2>&1 || exit $?
done
cat ${T}_timeline.log | grep -v amdgpu.ids
for v in "0 0" "1 1"; do
  set -- $v
  timeout -k 10 300 python -u bench.py --model resnet50 --emulate-world 8 --emulate-only 0,3,5 --steps 2 --warmup 1 \
    --search-pl $1 --search-spread $2 > ${T}_emu50_pl$1_sp$2.json 2> ${T}_emu50_pl$1_sp$2.err || exit $?
  python - ${T}_emu50_pl$1_sp$2.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[1], "shard ms", [round(x, 2) for x in d["shard_ms_per_sweep"]], [ {k: v for k, v in s.items() if k in ("gemm", "search")} for s in d["shard_kernel_avg_us"]])
PY
done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > ${T}_bench_r18.json 2> ${T}_bench_r18.err || exit $?
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r05b_bench_r18.json") if l.startswith("{")][-1])
print("C3 value", round(d["value"]), "ms/step", round(d["ms_per_step"], 2), {k: round(v["launch_avg_us"], 2) for k, v in d.get("roofline_kernels", {}).items()})
PY
timeout -k 10 300 python -u tools/epc_profile.py > ${T}_epc_profile.log 2>&1; cat ${T}_epc_profile.log | grep -v amdgpu.ids
