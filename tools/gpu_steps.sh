#!/bin/bash
# Run GPU steps in order; stop at the first step that crashed/faulted/timed out (exit not 0/1).
# usage: tools/gpu_steps.sh "<name>:<timeout>:<cmd>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; to="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] $cmd (timeout ${to}s)" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: step $name exited with $rc" | tee -a gpurun_out/steps.log
    exit $rc
  fi
done
