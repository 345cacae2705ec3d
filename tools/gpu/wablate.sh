#!/bin/bash
# halo wgrad ablations (PCA_HALO_ABLATE: 1 = no DMA, 2 = no MFMA phase, 4 = no epilogue)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
export PCA_TUNE_CACHE=/tmp/wab.json
for b in 1024 128; do
for shp in "64 64 32" "256 256 8"; do
  set -- $shp
  for ab in 0 1 2 4 6 7; do
    PCA_HALO_ABLATE=$ab timeout -k 10 120 python tools/time_conv.py --batch $b --cin $1 --cout $2 --h $3 --passes wgrad --tag "ab$ab" || exit 1
  done
done
done
