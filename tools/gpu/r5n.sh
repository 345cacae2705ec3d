#!/bin/bash
# SimpleDLA zero-copy Root: numerics vs the copying concat + SimpleDLA bs256 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5n; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_zero_copy_cat_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -14 $O/pytest.log; [ $rc = 0 ] || exit 1
for m in SimpleDLA DLA; do for rep in 1 2; do for Z in 1 0; do
  PCA_ZERO_COPY_CAT=$Z timeout -k 10 300 python bench.py --model $m --batch 256 --steps 15 --warmup 5 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('zc=$Z $m b256', d['ms_per_step'])" || exit 1
done; done; done
