#!/bin/bash
# depthwise BN-epilogue fusion: numerics, model-level tests, same-box A/B on the mobile benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_production_gpu.py tests/test_ops_gpu.py -k "depthwise or MobileNetV2 or EfficientNet or zoo" -x -q --timeout 300 --timeout-method thread 2>&1 | tail -40
rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
for m in "EfficientNetB0 128" "MobileNetV2 1024" "MobileNetV2 128"; do
  set -- $m
  for arm in 0 1 0 1; do
    PCA_DW_BN_FUSE=$arm timeout -k 10 200 python bench.py --model $1 --batch $2 --steps 20 --warmup 5 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1 b$2 fuse=$arm', d['ms_per_step'])" || exit 1
  done
done
