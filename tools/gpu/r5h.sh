#!/bin/bash
# kernel timelines of the concat-heavy models at bs256 (DPN26, ShuffleNetV2, SimpleDLA, DLA)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for m in ${MODELS:-DPN26 ShuffleNetV2_1 SimpleDLA DLA}; do
  BENCH_ARGS="--model $m" bash tools/gpu/prof_bench.sh r5h_$m 256 || exit 1
done
