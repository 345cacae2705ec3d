#!/bin/bash
# igemm register-pipelined K loop: numerics (every tile config) + same-box A/B of PCA_IGEMM_ILV
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ilv
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "tile_config or fwd_dgrad_wgrad or group_padded or channel_shuffle or chan_remap" > gpurun_out/ilv/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/ilv/pytest.log; [ $rc = 0 ] || exit 1
bash tools/gpu/ab_env.sh "PCA_IGEMM_ILV=0" "PCA_IGEMM_ILV=1" 1024 128
