#!/bin/bash
# GPU suite (incl. robust-BN and depthwise-BN-fusion tests), candidate numerics, tune logs, traces
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4d
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4d/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4d/pytest.log; grep -E "^FAILED|^ERROR" gpurun_out/r4d/pytest.log | head -30
[ $rc -gt 1 ] && exit $rc
for b in 1024 128; do
  PCA_TUNE_LOG=1 timeout -k 10 300 python bench.py --batch $b --steps 20 --warmup 5 \
    > gpurun_out/r4d/tune_b$b.json 2> gpurun_out/r4d/tune_b$b.log || exit 1
  cat gpurun_out/r4d/tune_b$b.json
done
bash tools/gpu/prof_bench.sh r4d 1024 || exit 1
timeout -k 10 400 python -u tools/diag/cand_check.py --batch 1024 --skip-wgrad > gpurun_out/r4d/cand1024.log 2>&1; rc=$?
tail -2 gpurun_out/r4d/cand1024.log; grep BAD gpurun_out/r4d/cand1024.log | head -30
exit 0
