#!/bin/bash
# Same-box A/B of two source trees (each a directory holding bench.py + a built
# pytorch_cifar_amd/): ab_tree.sh <dirA> <dirB> [batches...]; env ENV_A / ENV_B per arm.
# Each arm tunes once into its own cache, then 3 interleaved reps per batch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
A=$1; B=$2; shift 2
BS=${@:-1024 128}
for arm in A B; do
  D=$([ $arm = A ] && echo "$A" || echo "$B"); E=$([ $arm = A ] && echo "$ENV_A" || echo "$ENV_B")
  for b in $BS; do
    env $E PCA_TUNE_CACHE=/tmp/tune_tree_$arm.json timeout -k 10 300 python $D/bench.py --batch $b --steps 5 --warmup 3 > /dev/null 2>&1 || { echo "arm $arm b$b failed"; exit 1; }
  done
done
for rep in 1 2 3; do
  for arm in A B; do
    D=$([ $arm = A ] && echo "$A" || echo "$B"); E=$([ $arm = A ] && echo "$ENV_A" || echo "$ENV_B")
    for b in $BS; do
      env $E PCA_TUNE_CACHE=/tmp/tune_tree_$arm.json timeout -k 10 300 python $D/bench.py --batch $b --steps 30 --warmup 10 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$arm [$D $E] b$b', d['ms_per_step'])" || exit 1
    done
  done
done
