#!/bin/bash
# halo wgrad: XCD-aware block order on / off, per layer geometry (autotuned per arm)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for b in 1024 128; do
for shp in "64 64 32" "128 128 16" "256 256 8" "512 512 4"; do
  set -- $shp
  for x in 0 1; do
    PCA_HALO_XCD=$x timeout -k 10 120 python tools/time_conv.py --batch $b --cin $1 --cout $2 --h $3 --passes wgrad --tag "xcd$x" || exit 1
  done
done
done
