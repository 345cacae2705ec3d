#!/bin/bash
# epilogue VALU diet (pack2 as one cvt_pk, scalar c64 sums, single-rounding addend) vs HEAD~ tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_production_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc = 0 ] || exit 1
for rep in 1 2; do for T in cur base; do for P in fwd dgrad; do
  S=tools/conv_one.py; [ $T = base ] && S=ab/base/conv_one.py
  timeout -k 10 60 python $S --pass $P --iters 20 2>&1 | tail -1 | sed "s|^|$T |" || exit 1
done; done; done
bash tools/gpu/ab_tree.sh . ab/base 1024 128 || exit 1
