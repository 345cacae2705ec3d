#!/bin/bash
# Full GPU suite, then the whole-zoo native-vs-stock table at bs256 (one line per model).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/final/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 1000 python -u tools/zoo_bench.py --batch 256 --steps 10 --warmup 3 --timeout 120 | tee gpurun_out/final/zoo_bs256_r2.jsonl
