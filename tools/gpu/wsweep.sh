#!/bin/bash
# wgrad candidate sweeps at the bs128 shard's 3x3 s1 geometries
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for shp in "512 512 4" "256 256 8" "128 128 16" "64 64 32"; do
  set -- $shp
  timeout -k 10 120 python tools/wgrad_sweep.py --batch ${B:-128} --cin $1 --cout $2 --h $3 --top 8 || exit 1
done
