#!/bin/bash
# row-staged channel remap: numerics, then the odd-width grouped nets at bs256
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/remap2
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "group_padded or channel_shuffle or chan_remap or zoo_matches" > gpurun_out/remap2/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/remap2/pytest.log; [ $rc = 0 ] || exit 1
for m in DPN26 RegNetX_200MF RegNetY_400MF ShuffleNetG2 ShuffleNetG3 ResNeXt29_32x4d PNASNetA densenet_cifar LeNet; do
  timeout -k 10 150 python bench.py --model $m --batch 256 --steps 10 --warmup 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$m', d['ms_per_step'], d['value'])" || exit 1
done
