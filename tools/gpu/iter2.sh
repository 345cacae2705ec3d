#!/bin/bash
# Focused check + bench: pytest -k <expr>, then ResNet-18 / MobileNetV2 / EfficientNet-B0 benches
# and zoo timelines. usage: bash tools/gpu/iter2.sh <tag> <pytest -k expr>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
tag=$1; k=$2
mkdir -p gpurun_out/it
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$k" > gpurun_out/it/${tag}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/it/${tag}_pytest.log
[ $rc -ne 0 ] && exit $rc
for spec in "ResNet18 1024" "ResNet18 128" "MobileNetV2 1024" "MobileNetV2 128" "EfficientNetB0 1024" "EfficientNetB0 128"; do
  set -- $spec
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --model $1 --batch $2 > gpurun_out/it/${tag}_$1_b$2.json 2>gpurun_out/it/${tag}_$1_b$2.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/it/${tag}_$1_b$2.json').read().strip().splitlines()[-1]); print('$1 b$2 %.3f ms %.1f img/s' % (d['ms_per_step'], d['value']))"
done
bash tools/gpu/prof_zoo.sh $tag
