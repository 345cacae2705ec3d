#!/bin/bash
# split-K reduce grid cap A/B at the shard sizes, then the native zoo pass
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu/ab_env.sh "PCA_SPLITK_RED_CAP=512" "PCA_SPLITK_RED_CAP=128" 128 256 || exit 1
bash tools/gpu/zoo_r3.sh
