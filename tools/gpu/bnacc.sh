#!/bin/bash
# A/B of PCA_BN_ACC_MAX_ELEMS (separate BN-backward reduce into the sharded accumulator, no
# finalize launch) per model / batch, same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ba
for round in 1 2; do for v in 0 1048576 4194304 33554432; do
  for spec in "EfficientNetB0 128" "EfficientNetB0 1024" "MobileNetV2 128" "MobileNetV2 1024" "ResNet18 128" "ResNet18 1024"; do
    set -- $spec
    PCA_BN_ACC_MAX_ELEMS=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --model $1 --batch $2 > gpurun_out/ba/o.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/ba/o.json').read().strip().splitlines()[-1]); print('$round max=$v $1 b$2 %.3f ms' % d['ms_per_step'])"
  done
done; done
