#!/bin/bash
# same-box A/B of an env knob on model benches: ab_model.sh "<envA>" "<envB>" "Model batch" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
A=$1; B=$2; shift 2
for mb in "$@"; do
  set -- $mb
  for rep in 1 2; do
    for arm in A B; do
      E=$([ $arm = A ] && echo "$A" || echo "$B")
      env $E timeout -k 10 200 python bench.py --model $1 --batch $2 --steps 20 --warmup 5 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$arm [$E] $1 b$2', d['ms_per_step'])" || exit 1
    done
  done
done
