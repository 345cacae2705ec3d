#!/bin/bash
# Kernel-trace timelines of the MobileNetV2 / EfficientNet-B0 bench steps (BASELINE configs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
tag=$1
BENCH_ARGS="--model MobileNetV2" bash tools/gpu/prof_bench.sh ${tag}_mnv2 1024 128 || exit 1
BENCH_ARGS="--model EfficientNetB0" bash tools/gpu/prof_bench.sh ${tag}_effb0 1024 128 || exit 1
