#!/bin/bash
# ShuffleNetV2 stages on SplitBlock halves: GPU tests, then same-box A/B against the
# block-by-block join + split (PCA_ZERO_COPY_CAT=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_zero_copy_cat_gpu.py -k "shuffle or interleave" > gpurun_out/r5t_tests.log 2>&1 || { tail -30 gpurun_out/r5t_tests.log; exit 1; }
tail -3 gpurun_out/r5t_tests.log
bash tools/gpu/ab_model.sh "PCA_ZERO_COPY_CAT=1" "PCA_ZERO_COPY_CAT=0" "ShuffleNetV2_0.5 256" "ShuffleNetV2_1 256" "ShuffleNetV2_2 256"
