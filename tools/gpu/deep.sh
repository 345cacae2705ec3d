#!/bin/bash
# deep-ring halo wgrad configs: numerics, then bench at the shard sizes and bs1024 (autotuned)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/deep
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "wgrad" > gpurun_out/deep/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/deep/pytest.log; [ $rc = 0 ] || exit 1
for rep in 1 2; do
  for b in 128 256 1024; do
    timeout -k 10 200 python bench.py --batch $b --steps 30 --warmup 10 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('b$b', d['ms_per_step'])" || exit 1
  done
done
PCA_CONV_VERBOSE=1 timeout -k 10 200 python bench.py --batch 128 --steps 2 --warmup 1 > gpurun_out/deep/verbose128.log 2>&1
grep -c "halo wgrad" gpurun_out/deep/verbose128.log
