#!/bin/bash
# zero-copy concat: numerics (bitwise vs the copying concat), GoogLeNet bench A/B, trace check.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_zero_copy_cat_gpu.py tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread -k "zero_copy or slab or strided or GoogLeNet or inception" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc = 0 ] || exit 1
for rep in 1 2; do for Z in 1 0; do
  PCA_ZERO_COPY_CAT=$Z timeout -k 10 300 python bench.py --model GoogLeNet --batch 256 --steps 10 --warmup 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('zc=$Z GoogLeNet b256', d['ms_per_step'])" || exit 1
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --model GoogLeNet --batch 256 --steps 5 --warmup 3 > $O/prof.log 2>&1 || exit 1
f=$(ls $O/prof/*kernel_stats.csv $O/prof/*/*kernel_stats.csv 2>/dev/null | head -1)
grep -c "cat_nhwc\|split_nhwc" "$f" || true
