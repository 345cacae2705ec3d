#!/bin/bash
# stem forward kernel: numerics, then same-box A/B against the generic igemm (PCA_STEM_FWD=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sf
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "conv_fwd_dgrad or zoo or accumulators or resnet18 or weight_prep or graph" > gpurun_out/sf/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/sf/pytest.log
[ $rc -ne 0 ] && exit $rc
for round in 1 2; do for v in 1 0; do for spec in "ResNet18 1024" "ResNet18 128" "MobileNetV2 1024"; do
  set -- $spec
  PCA_STEM_FWD=$v timeout -k 10 300 python bench.py --steps 30 --warmup 10 --model $1 --batch $2 > gpurun_out/sf/o.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/sf/o.json').read().strip().splitlines()[-1]); print('$round stem=$v $1 b$2 %.3f ms' % d['ms_per_step'])"
done; done; done
bash tools/gpu/prof_bench.sh sf 1024 128
