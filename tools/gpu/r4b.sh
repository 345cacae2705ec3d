#!/bin/bash
# Diagnose the ResNet-18 bs1024 production-step mismatch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4b
timeout -k 10 300 python -u tools/diag/prod_layers.py --batch 1024 > gpurun_out/r4b/default.log 2>&1 || exit $?
tail -40 gpurun_out/r4b/default.log
PCA_BN_ACC=0 timeout -k 10 300 python -u tools/diag/prod_layers.py --batch 1024 > gpurun_out/r4b/noacc.log 2>&1 || exit $?
PCA_CONV_AUTOTUNE=0 timeout -k 10 300 python -u tools/diag/prod_layers.py --batch 1024 > gpurun_out/r4b/notune.log 2>&1 || exit $?
grep "logits" gpurun_out/r4b/*.log
timeout -k 10 300 python -u -m pytest tests/test_production_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4b/prod.log 2>&1; tail -3 gpurun_out/r4b/prod.log
