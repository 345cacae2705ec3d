#!/bin/bash
# What the driver runs at round end: the GPU suite, smoke(), and bench.py with default arguments.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/end
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/end/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/end/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/end/smoke.log 2>&1 || { tail -20 gpurun_out/end/smoke.log; exit 1; }
tail -1 gpurun_out/end/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/end/bench.json 2>gpurun_out/end/bench.err || { tail -20 gpurun_out/end/bench.err; exit 1; }
cat gpurun_out/end/bench.json
timeout -k 10 300 python bench.py --batch 128 > gpurun_out/end/bench_b128.json 2>/dev/null || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/end/bench_b128.json').read().strip().splitlines()[-1]); print('b128 %.3f ms %.1f img/s' % (d['ms_per_step'], d['value']))"
