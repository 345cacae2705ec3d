#!/bin/bash
# every autotune candidate's numerics at the production shapes (bs1024, bs128)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4c
timeout -k 10 500 python -u tools/diag/cand_check.py --batch 1024 > gpurun_out/r4c/b1024.log 2>&1; rc=$?
tail -3 gpurun_out/r4c/b1024.log; grep BAD gpurun_out/r4c/b1024.log | head -30
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u tools/diag/cand_check.py --batch 128 > gpurun_out/r4c/b128.log 2>&1; rc=$?
tail -3 gpurun_out/r4c/b128.log; grep BAD gpurun_out/r4c/b128.log | head -30
exit 0
