#!/bin/bash
# c64 kernel check: numerics (conv kernel tests + ResNet-18 zoo / fusion tests), per-pass timing,
# and the bench step at bs1024 / bs128.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_ops_gpu.py -k "conv or resnet18 or ResNet18 or bn_backward_reduce" -x -q --timeout 200 --timeout-method thread > gpurun_out/r3/c64_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3/c64_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/r3/c64_tests.log | head -20; exit $rc; }
for b in 1024 128; do
  timeout -k 10 120 python tools/time_conv.py --batch $b --cin 64 --cout 64 --h 32 || exit 1
done
timeout -k 10 200 python bench.py > gpurun_out/r3/bench_b1024.json 2>&1 || { tail -5 gpurun_out/r3/bench_b1024.json; exit 1; }
tail -n 1 gpurun_out/r3/bench_b1024.json
timeout -k 10 200 python bench.py --batch 128 > gpurun_out/r3/bench_b128.json 2>&1 || exit 1
tail -n 1 gpurun_out/r3/bench_b128.json
