#!/bin/bash
# Quick GPU iteration: kernel tests matching $1 (pytest -k), then the bs128 / bs1024 benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/q
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$1" > gpurun_out/q/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/q/pytest.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
[ $rc -ne 0 ] && exit 1
for b in 128 1024; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 10 --batch $b > gpurun_out/q/r18_b$b.json 2>gpurun_out/q/r18_b$b.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/q/r18_b$b.json').read().strip().splitlines()[-1]); print('b$b %.3f ms %.1f img/s' % (d['ms_per_step'], d['value']))"
done
