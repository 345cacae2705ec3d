#!/bin/bash
# odd-width convs: padded statistics read in place by the BN finalize (no stats unpad). GPU tests, then a
# same-box A/B against the round's previous commit (ab/base) on the odd-width zoo models
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ops_gpu.py tests/test_fused_sgd_gpu.py tests/test_bn_robust_gpu.py tests/test_bn_shift_gpu.py -k "padded or group or fused or bn" > gpurun_out/r5y_tests.log 2>&1 || { tail -40 gpurun_out/r5u_tests.log; exit 1; }
tail -3 gpurun_out/r5y_tests.log
for rep in 1 2; do
  for m in "ShuffleNetV2_1 256" "PNASNetA 256" "ShuffleNetG2 256"; do
    set -- $m
    for arm in new base; do
      d=.; [ $arm = base ] && d=ab/base
      (cd $d && timeout -k 10 200 python bench.py --model $1 --batch $2 --steps 20 --warmup 5 2>/dev/null) | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$arm $1 b$2', d['ms_per_step'])" || exit 1
    done
  done
done
