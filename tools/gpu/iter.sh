#!/bin/bash
# Iteration check: full GPU test suite, ResNet-18 bench at bs1024 / bs128, kernel-trace timeline
# of both. usage: bash tools/gpu/iter.sh <tag> [pytest -k expr]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
tag=$1; k=${2:-}
mkdir -p gpurun_out/it
if [ -n "$k" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$k" > gpurun_out/it/${tag}_pytest.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/it/${tag}_pytest.log 2>&1
fi
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/it/${tag}_pytest.log
[ $rc -ne 0 ] && exit $rc
for b in 1024 128; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 10 --batch $b > gpurun_out/it/${tag}_b$b.json 2>gpurun_out/it/${tag}_b$b.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/it/${tag}_b$b.json').read().strip().splitlines()[-1]); print('b$b %.3f ms %.1f img/s' % (d['ms_per_step'], d['value']))"
done
bash tools/gpu/prof_bench.sh $tag 1024 128
