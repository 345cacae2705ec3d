#!/bin/bash
# same-box A/B of the layer-1 c64 kernel versions (PCA_C64_V=1 round 2, 2 current)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for rep in 1 2; do
for v in 1 2; do
  for b in 1024 128; do
    PCA_C64_V=$v timeout -k 10 120 python tools/time_conv.py --batch $b --cin 64 --cout 64 --h 32 --passes fwd,dgrad,dgrad_bn | sed "s/^/v$v /" || exit 1
  done
done
done
