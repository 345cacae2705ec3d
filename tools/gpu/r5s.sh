#!/bin/bash
# fused BN-reduce epilogues: istd applied at the flush, bit-select mask — numerics + A/B vs ab/base
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5s; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_ops_gpu.py tests/test_production_gpu.py tests/test_bn_shift_gpu.py -x -q --timeout 300 --timeout-method thread -k "dgrad or bn or BN or c64 or halo or production or resnet18 or dual" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc = 0 ] || exit 1
bash tools/gpu/ab_tree.sh ab/base . 1024 128
