#!/bin/bash
# Run GPU steps in order, each under its own time limit; a step that fails normally (rc 1: a test
# or assertion failure) does not stop the chain, anything else (fault, abort, timeout) does.
#   bash tools/gpu/steps.sh <seconds> '<cmd>' [<seconds> '<cmd>']...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
while [ $# -ge 2 ]; do
  t=$1; c=$2; shift 2
  echo "=== [$t s] $c"
  timeout -k 10 "$t" bash -c "$c"
  rc=$?
  echo "=== rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
