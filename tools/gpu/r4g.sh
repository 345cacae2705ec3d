#!/bin/bash
# graph == eager test under knobs (which change broke bitwise equality), then the production tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4g
for env in "PCA_BN_SHIFT=1" "PCA_BN_SHIFT=0" "PCA_HX_ILV=0"; do
  env $env timeout -k 10 200 python -u -m pytest tests/test_cli_gpu.py -q -k graph_steps_equal --timeout 150 --timeout-method thread > gpurun_out/r4g/graph.log 2>&1
  echo "$env: $(tail -1 gpurun_out/r4g/graph.log)"
done
timeout -k 10 900 python -u -m pytest tests/test_production_gpu.py tests/test_dw_bn_fuse_gpu.py -v --timeout 400 --timeout-method thread > gpurun_out/r4g/prod.log 2>&1
rc=$?; echo "prod rc=$rc"; grep -E "PASS|FAIL|Error" gpurun_out/r4g/prod.log | head -30
