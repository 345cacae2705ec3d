#!/bin/bash
# PMC step tables (MFMA busy %, traffic past L2) for the BASELINE configs: ResNet-18 bs1024,
# MobileNetV2 bs1024, EfficientNet-B0 bs128 (the 8-GPU shard)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu/pmc_step.sh r18 1024 || exit 1
BENCH_ARGS="--model MobileNetV2" bash tools/gpu/pmc_step.sh mnv2 1024 || exit 1
BENCH_ARGS="--model EfficientNetB0" bash tools/gpu/pmc_step.sh effb0 128
