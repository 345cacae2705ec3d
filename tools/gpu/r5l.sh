#!/bin/bash
# shipped tune table vs tuning afresh, same box, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for rep in 1 2 3; do for T in 1 0; do for b in 1024 128; do
  PCA_TUNE_TABLE=$T PCA_TUNE_CACHE=/tmp/tc_$T.json timeout -k 10 200 python bench.py --batch $b --steps 30 --warmup 10 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('table=$T b$b', d['ms_per_step'], d['config']['kernel_selection'])" || exit 1
done; done; done
