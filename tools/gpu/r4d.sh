#!/bin/bash
# GPU suite (incl. the robust-BN test), candidate numerics sweep, tune logs, step traces
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4d
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4d/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4d/pytest.log; grep -E "^FAILED|Error" gpurun_out/r4d/pytest.log | head -20
[ $rc -gt 1 ] && exit $rc
timeout -k 10 500 python -u tools/diag/cand_check.py --batch 1024 > gpurun_out/r4d/cand1024.log 2>&1; rc=$?
tail -2 gpurun_out/r4d/cand1024.log; grep BAD gpurun_out/r4d/cand1024.log | head -30
[ $rc -gt 1 ] && exit $rc
for b in 1024 128; do
  PCA_TUNE_LOG=1 timeout -k 10 300 python bench.py --batch $b --steps 20 --warmup 5 \
    > gpurun_out/r4d/tune_b$b.json 2> gpurun_out/r4d/tune_b$b.log || exit 1
  cat gpurun_out/r4d/tune_b$b.json
done
bash tools/gpu/prof_bench.sh r4d 1024 128
timeout -k 10 300 python -u tools/winograd_ab.py --batch 1024 > gpurun_out/r4d/winograd.jsonl 2>&1; cat gpurun_out/r4d/winograd.jsonl | tail -4
