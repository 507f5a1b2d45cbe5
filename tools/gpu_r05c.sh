#!/bin/bash
# Round 5 session c: the GPU test files not yet run on this tree (EPC solves first), the
# horizon tests against F11, then the search-form A/B, the EPC profile and a C3 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=gpurun_out/r05c
timeout -k 10 900 python -u -m pytest tests/test_gpu_epc.py tests/test_gpu_panel.py tests/test_gpu_parity.py \
  tests/test_gpu_reference.py tests/test_torch_ops.py tests/test_gpu_horizon.py -x -q -rf -s --timeout 300 \
  --timeout-method thread > ${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "C2 |C3 |parafac-epc|passed|failed|Error" ${T}_pytest.log | tail -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc   # 1 = a test assertion failed: the diagnostics below still run
timeout -k 10 300 python -u tools/epc_profile.py > ${T}_epc_profile.log 2>&1; rc=$?; grep -v amdgpu.ids ${T}_epc_profile.log; [ $rc -ne 0 ] && exit $rc
for g in 36 144 256 432 708; do
  for m in 0 1; do timeout -k 5 60 tools/probes/barrier_probe $m $g 999 >> ${T}_barrier_probe.log 2>&1 || exit $?; done
done
cat ${T}_barrier_probe.log
for v in "0 0" "0 1" "2 0" "2 1"; do
  set -- $v
  echo "== timeline lone layer4 pl=$1 spread=$2" >> ${T}_timeline.log
  ADMMQ_LIB=$PWD/tools/tracelib/libadmmq.so timeout -k 10 120 python -u tools/hist_timeline.py --shapes 512:1141 \
    --iters 6 --pl $1 --spread $2 >> ${T}_timeline.log 2>&1 || exit $?
done
grep -v amdgpu.ids ${T}_timeline.log
for v in "0 0" "1 1"; do
  set -- $v
  timeout -k 10 300 python -u bench.py --model resnet50 --emulate-world 8 --emulate-only 0,3,5 --steps 2 --warmup 1 \
    --search-pl $1 --search-spread $2 > ${T}_emu50_pl$1_sp$2.json 2> ${T}_emu50_pl$1_sp$2.err || exit $?
  python - ${T}_emu50_pl$1_sp$2.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[1], "shard ms", [round(x, 2) for x in d["shard_ms_per_sweep"]], [{k: v for k, v in s.items() if k in ("gemm", "search")} for s in d["shard_kernel_avg_us"]])
PY
done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > ${T}_bench_r18.json 2> ${T}_bench_r18.err || exit $?
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r05c_bench_r18.json") if l.startswith("{")][-1])
print("C3 value", round(d["value"]), "ms/step", round(d["ms_per_step"], 2), {k: round(v["launch_avg_us"], 2) for k, v in d.get("roofline_kernels", {}).items()})
PY
