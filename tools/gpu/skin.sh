#!/bin/bash
# split-K in-kernel finish: numerics, production step, then same-box A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/skin
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_ops_gpu.py tests/test_production_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "splitk or tile_config or fwd_dgrad_wgrad or dual or reduce_fusion or production or trajectory" > gpurun_out/skin/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/skin/pytest.log; [ $rc = 0 ] || exit 1
bash tools/gpu/ab_env.sh "PCA_SPLITK_INKERNEL=0" "PCA_SPLITK_INKERNEL=1" 128 256
