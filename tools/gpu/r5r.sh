#!/bin/bash
# packed ReLU-mask stores: BN tests, bn_bench both trees, same-box A/B vs ab/base
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_ops_gpu.py tests/test_bn_shift_gpu.py tests/test_zero_copy_cat_gpu.py -x -q --timeout 300 --timeout-method thread -k "bn or BN or batchnorm or resnet18 or slab or mask" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc = 0 ] || exit 1
for d in ab/base .; do echo "== $d"; timeout -k 10 200 python $d/tools/bn_bench.py 2>/dev/null | head -9 || exit 1; done
bash tools/gpu/ab_tree.sh ab/base . 1024 128
