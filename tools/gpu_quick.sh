#!/bin/bash
# GPU tests (all, or the given pytest args), then a short C3 bench line.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
if [ $# -eq 0 ]; then set -- tests -m gpu; fi
timeout -k 10 900 python -u -m pytest "$@" -x -q -rf --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/bench.log") if l.startswith("{")][-1])
print("value", round(d["value"]), "ms/step", round(d["ms_per_step"], 2), "step frac", round(d["step_roofline"]["frac"], 3))
for k, v in d.get("roofline_kernels", {}).items():
    print(k, "avg_us", round(v["launch_avg_us"], 2), v["bound"], "frac", round(v["frac"], 3))
print("ms/step by kernel", {k: round(v, 2) for k, v in d["kernel_ms_per_step"].items()})
PY
