#!/bin/bash
# -fno-slp-vectorize tree (ab/nosl) vs default: per-call c64 timing, then the bench A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for rep in 1 2; do for T in tools ab/nosl; do for V in 2 4; do for P in fwd dgrad; do
  PCA_C64_V=$V timeout -k 10 60 python $T/conv_one.py --pass $P --iters 20 2>&1 | tail -1 | sed "s|^|$T v$V |" || exit 1
done; done; done; done
bash tools/gpu/ab_tree.sh . ab/nosl 1024 128 || exit 1
