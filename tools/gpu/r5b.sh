#!/bin/bash
# c64 v3 (32x32x16) check: numerics, same-box A/B vs v2, kernel trace of the bs1024 step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "c64 or conv_fwd_dgrad_wgrad or halo_kernel" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc = 0 ] || exit 1
bash tools/gpu/ab_env.sh "PCA_C64_V=2" "PCA_C64_V=3" 1024 128 || exit 1
bash tools/gpu/prof_bench.sh r5b 1024 || exit 1
