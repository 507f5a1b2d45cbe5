#!/bin/bash
# C4 / C5 bench lines, and the rocprofv3 kernel-trace
# stats of the EPC initialiser on layer1.0.conv1 (tools/epc_profile.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=gpurun_out/${1:-c4c5_epc}
export TMPDIR=/tmp
for m in resnet50 llama7b; do
  timeout -k 10 400 python -u bench.py --model $m --steps 3 --warmup 1 --no-cpu-baseline > ${T}_bench_$m.json 2> ${T}_bench_$m.err || { tail ${T}_bench_$m.err; exit 5; }
  python3 - ${T}_bench_$m.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[1], round(d["value"]), "ms", round(d["ms_per_step"], 1), "frac", round(d["roofline"]["frac"], 3))
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${T}_epc_ktrace -o run -- python3 tools/epc_profile.py > ${T}_epc_ktrace.log 2>&1 || { tail ${T}_epc_ktrace.log; exit 6; }
echo epc ktrace done
