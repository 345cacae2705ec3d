#!/bin/bash
# grouped convs as block-diagonal super-groups: numerics + DPN26 / ResNeXt29_32x4d A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r5i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread -k "group_padded or direct_conv" > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log; [ $rc = 0 ] || exit 1
for mb in "DPN26 256" "ResNeXt29_32x4d 256" "RegNetX_200MF 256"; do set -- $mb
for rep in 1 2; do for Z in 1 all 0; do
  PCA_GROUP_DENSE=$Z timeout -k 10 300 python bench.py --model $1 --batch $2 --steps 10 --warmup 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('gd=$Z $1 b$2', d['ms_per_step'])" || exit 1
done; done; done
