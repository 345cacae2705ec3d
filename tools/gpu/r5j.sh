#!/bin/bash
# igemm epilogue prefetch: conv numerics, then same-box A/B vs the HEAD tree (ab/base)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread -k "dgrad or igemm or conv" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc = 0 ] || exit 1
bash tools/gpu/ab_tree.sh ab/base . 1024 128
