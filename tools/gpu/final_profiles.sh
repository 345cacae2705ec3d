#!/bin/bash
# Final-tree kernel traces (ResNet-18 bs1024 / bs128, EfficientNet-B0 bs128, MobileNetV2 bs1024) and the ResNet-18 PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu/prof_bench.sh r5f_r18 1024 128 && bash tools/gpu/pmc_step.sh r5f 1024 128 && BENCH_ARGS="--model EfficientNetB0" bash tools/gpu/prof_bench.sh r5f_effb0 128 && BENCH_ARGS="--model MobileNetV2" bash tools/gpu/prof_bench.sh r5f_mnv2 1024
