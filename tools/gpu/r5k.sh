#!/bin/bash
# BN row kernels: rows in flight (PCA_BN_U) x grid cap (PCA_BN_ROWS_CAP), microbench + step A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for u in 4 8; do for cap in 512 1024 2048; do
  echo "U=$u cap=$cap"
  PCA_BN_U=$u PCA_BN_ROWS_CAP=$cap timeout -k 10 200 python tools/bn_bench.py 2>/dev/null | grep -E "apply|bwd" | grep -E "32x32|16x16" || exit 1
done; done
for rep in 1 2; do for E in "PCA_BN_U=4" "PCA_BN_U=8" "PCA_BN_U=8 PCA_BN_ROWS_CAP=1024"; do for b in 1024 128; do
  env $E timeout -k 10 200 python bench.py --batch $b --steps 30 --warmup 10 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[$E] b$b', d['ms_per_step'])" || exit 1
done; done; done
