#!/bin/bash
# round-3c: fresh ResNet-18 step profiles (bs1024 / bs128) + side-stream wgrad A/B at bs128
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
export PCA_TUNE_CACHE=/tmp/tune_prof.json
for b in 1024 128; do
  timeout -k 10 200 python bench.py --batch $b --steps 5 --warmup 3 > /dev/null 2>&1 || exit 1
done
bash tools/gpu/prof_bench.sh r3c 1024 128 || exit 1
unset PCA_TUNE_CACHE
bash tools/gpu/ab_env.sh "PCA_WGRAD_STREAM=0" "PCA_WGRAD_STREAM=1" 128
