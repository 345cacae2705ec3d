#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4h
timeout -k 10 200 python -u tools/diag/graph_eager.py > gpurun_out/r4h/ge.log 2>&1; rc=$?
echo "graph_eager rc=$rc"; grep step gpurun_out/r4h/ge.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/r4e.sh
