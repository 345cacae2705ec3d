#!/bin/bash
# BASELINE configs 4/5 (MobileNetV2, EfficientNet-B0) at bs1024 and the bs128 shard
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/zf
for spec in "MobileNetV2 1024" "MobileNetV2 128" "EfficientNetB0 1024" "EfficientNetB0 128"; do
  set -- $spec
  timeout -k 10 300 python bench.py --steps 30 --warmup 10 --model $1 --batch $2 > gpurun_out/zf/$1_b$2.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/zf/$1_b$2.json').read().strip().splitlines()[-1]); print('$1 b$2 %.3f ms %.1f img/s' % (d['ms_per_step'], d['value']))"
done
