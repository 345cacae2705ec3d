#!/bin/bash
# compact stride-2 shortcut addend: kernel numerics, model tests, same-box A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread -k "compact_s2 or resnet18 or s2_dgrad or production" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc = 0 ] || exit 1
for rep in 1 2 3; do for Z in 1 0; do for b in 1024 128; do
  PCA_S2C_ADDEND=$Z timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('s2c=$Z b$b', d['ms_per_step'])" || exit 1
done; done; done
