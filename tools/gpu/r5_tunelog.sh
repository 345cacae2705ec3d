#!/bin/bash
# Autotune trial log + bench of the headline shapes (bs1024 / bs128) on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5a; mkdir -p $O
for b in 1024 128; do
  PCA_TUNE_LOG=1 PCA_TUNE_CACHE=$O/tune_b$b.json timeout -k 10 200 python bench.py --batch $b --steps 30 --warmup 10 > $O/b$b.json 2> $O/tune_b$b.log || exit 1
  tail -1 $O/b$b.json
done
