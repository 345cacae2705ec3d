#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/dbg
PYTHONPATH=. timeout -k 10 200 python -u tools/probes/iter2_layers.py > gpurun_out/dbg/iter2.log 2>&1
echo rc=$?; tail -30 gpurun_out/dbg/iter2.log
