#!/usr/bin/env bash
# Run GPU steps in order on the gpurun box; each step has its own time limit.
# A test-failure exit (1) lets later steps run; a timeout, abort, segfault or any
# signal ends the script immediately (no further GPU work after a fault).
# usage: tools/gpu_run.sh "name|seconds|command" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/${name}.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc after $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/${name}.log"
  if grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|GPU fault|HSA_STATUS_ERROR|Error code 700" "gpurun_out/${name}.log"; then
    echo "=== stopping: step $name reported a GPU fault"
    exit 3
  fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping: step $name ended with rc=$rc"
    exit $rc
  fi
done
exit 0
