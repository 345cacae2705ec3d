#!/bin/bash
# Full GPU check: test suite, headline bench at the 1/2/4/8-GPU per-rank shards, BASELINE models,
# per-phase rocprofv3 step profiles. Writes under gpurun_out/rc/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/rc/pytest.log 2>&1
echo "pytest rc=$?"; tail -2 gpurun_out/rc/pytest.log
for b in 1024 512 256 128; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 10 --batch $b > gpurun_out/rc/r18_b$b.json 2>/dev/null || exit 1
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --model MobileNetV2 > gpurun_out/rc/mnv2.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --model EfficientNetB0 > gpurun_out/rc/effb0.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --model EfficientNetB0 --batch 128 > gpurun_out/rc/effb0_b128.json 2>/dev/null || exit 1
for f in gpurun_out/rc/*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('%-28s %8.3f ms %10.1f img/s' % ('$f'.split('/')[-1], d['ms_per_step'], d['value']))"; done
