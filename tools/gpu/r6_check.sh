#!/bin/bash
# Round-6 tree check: full GPU suite, smoke, default bench, the bs128 shard, and step traces of
# ResNet-18 bs1024/bs128, MobileNetV2 bs1024, EfficientNet-B0 bs128 (writes gpurun_out/r6c/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6c
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r6c/pytest.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/r6c/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6c/smoke.log 2>&1 || { echo smoke FAILED; tail -20 gpurun_out/r6c/smoke.log; exit 1; }
tail -1 gpurun_out/r6c/smoke.log
timeout -k 10 200 python bench.py > gpurun_out/r6c/b1024.json || exit 1
timeout -k 10 200 python bench.py --batch 128 --steps 50 --warmup 10 > gpurun_out/r6c/b128.json || exit 1
cat gpurun_out/r6c/*.json
bash tools/gpu/prof_bench.sh r6f_r18 1024 128 || exit 1
BENCH_ARGS="--model MobileNetV2" bash tools/gpu/prof_bench.sh r6f_mnv2 1024 || exit 1
BENCH_ARGS="--model EfficientNetB0" bash tools/gpu/prof_bench.sh r6f_effb0 128 || exit 1
