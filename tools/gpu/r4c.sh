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
for b in 1024 128; do
  PCA_TUNE_LOG=1 timeout -k 10 300 python bench.py --batch $b --steps 10 --warmup 5 \
    > gpurun_out/r4c/tune_b$b.json 2> gpurun_out/r4c/tune_b$b.log || exit 1
  cat gpurun_out/r4c/tune_b$b.json
done
bash tools/gpu/prof_bench.sh r4c 1024 128
