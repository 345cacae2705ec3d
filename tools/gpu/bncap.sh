#!/bin/bash
# BN row-kernel grid cap sweep (same box): bench step time at bs1024 / bs128
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
export PCA_TUNE_CACHE=/tmp/tune_bncap.json
timeout -k 10 200 python bench.py --steps 5 --warmup 3 > /dev/null 2>&1
timeout -k 10 200 python bench.py --batch 128 --steps 5 --warmup 3 > /dev/null 2>&1
for rep in 1 2; do
for cap in 2048 1024 512 4096; do
  for b in 1024 128; do
    PCA_BN_ROWS_CAP=$cap timeout -k 10 200 python bench.py --batch $b --steps 30 --warmup 10 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('cap $cap b$b', d['ms_per_step'])" || exit 1
  done
done
done
