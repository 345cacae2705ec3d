#!/bin/bash
# halo wgrad tap-row split: numerics + bench at bs128 / bs1024
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad" -x -q --timeout 300 --timeout-method thread 2>&1 | tail -3
rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --batch 128 > gpurun_out/r3/bench_b128.json 2>&1 || exit 1
tail -n 1 gpurun_out/r3/bench_b128.json
timeout -k 10 200 python bench.py > gpurun_out/r3/bench_b1024.json 2>&1 || exit 1
tail -n 1 gpurun_out/r3/bench_b1024.json
bash tools/gpu/prof_bench.sh r3b 1024 128
