#!/bin/bash
# dual-BN fused reduce + igemm register-pipelined K loop: numerics, then same-box A/Bs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ilv
timeout -k 10 500 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "dual or reduce_fusion" > gpurun_out/ilv/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/ilv/pytest.log; [ $rc = 0 ] || exit 1
bash tools/gpu/ab_env.sh "PCA_DUAL_BN_FUSE=0" "PCA_DUAL_BN_FUSE=1" 1024 128 || exit 1
bash tools/gpu/ab_env.sh "PCA_IGEMM_ILV=0" "PCA_IGEMM_ILV=1" 1024 128
