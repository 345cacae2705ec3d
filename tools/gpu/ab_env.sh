#!/bin/bash
# same-box A/B of an environment knob on the bench step: ab_env.sh "<envA>" "<envB>" [batches...]
# (each arm tunes once into its own cache, so a knob that changes the candidate set is honoured)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
A=$1; B=$2; shift 2
BS=${@:-1024 128}
for arm in A B; do
  E=$([ $arm = A ] && echo "$A" || echo "$B")
  for b in $BS; do
    env $E PCA_TUNE_CACHE=/tmp/tune_ab_$arm.json timeout -k 10 200 python bench.py --batch $b --steps 5 --warmup 3 > /dev/null 2>&1 || exit 1
  done
done
for rep in 1 2 3; do
  for arm in A B; do
    E=$([ $arm = A ] && echo "$A" || echo "$B")
    for b in $BS; do
      env $E PCA_TUNE_CACHE=/tmp/tune_ab_$arm.json timeout -k 10 200 python bench.py --batch $b --steps 30 --warmup 10 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$arm [$E] b$b', d['ms_per_step'])" || exit 1
    done
  done
done
