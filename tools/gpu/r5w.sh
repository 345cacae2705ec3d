#!/bin/bash
# kernel-trace timelines of the ShuffleNetV2 (halves path, plan-written padded operands) and
# DPN26 steps at bs256, final round-5 tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
BENCH_ARGS="--model ShuffleNetV2_0.5" bash tools/gpu/prof_bench.sh r5w_snv2_05 256 || exit 1
BENCH_ARGS="--model ShuffleNetV2_1" bash tools/gpu/prof_bench.sh r5w_snv2_1 256 || exit 1
BENCH_ARGS="--model DPN26" bash tools/gpu/prof_bench.sh r5w_dpn26 256 || exit 1
