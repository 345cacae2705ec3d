#!/bin/bash
# round-3 step profiles: ResNet-18 bs1024 / bs128, MobileNetV2 bs1024, EfficientNet-B0 bs128
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
export PCA_TUNE_CACHE=/tmp/tune_prof.json
for mb in "ResNet18 1024" "ResNet18 128" "MobileNetV2 1024" "EfficientNetB0 128"; do
  set -- $mb
  timeout -k 10 200 python bench.py --model $1 --batch $2 --steps 5 --warmup 3 > /dev/null 2>&1 || exit 1
  BENCH_ARGS="--model $1" bash tools/gpu/prof_bench.sh r3b_$1 $2 > /dev/null 2>&1 || exit 1
  timeout -k 10 200 python bench.py --model $1 --batch $2 --steps 30 --warmup 10 2>/dev/null | tail -1 > gpurun_out/prof/r3b_$1_b$2_bench.json || exit 1
  cat gpurun_out/prof/r3b_$1_b$2_bench.json
done
