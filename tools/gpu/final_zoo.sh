#!/bin/bash
# Full GPU suite, then the whole zoo at bs256 (one line per model): native only by default,
# with the stock comparator when STOCK=1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/final/pytest.log
[ $rc -ne 0 ] && exit $rc
NO=--native-only; [ "$STOCK" = 1 ] && NO=
timeout -k 10 1000 python -u tools/zoo_bench.py --batch 256 --steps 10 --warmup 3 --timeout 120 $NO | tee gpurun_out/final/zoo_bs256.jsonl
