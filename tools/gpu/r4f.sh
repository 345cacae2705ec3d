#!/bin/bash
# locate the MobileNetV2 bs1024 device fault (debug sync + op trace), then the graph==eager test
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4f
PCA_DEBUG_SYNC=1 PCA_DEBUG_TRACE=1 timeout -k 10 240 python -u tools/diag/mnv2_fault.py --model MobileNetV2 --batch 1024 > gpurun_out/r4f/mnv2.log 2> gpurun_out/r4f/mnv2.err
rc=$?; echo "mnv2 rc=$rc"; tail -5 gpurun_out/r4f/mnv2.log; grep -v "^Extension modules" gpurun_out/r4f/mnv2.err | tail -25 | cut -c1-250
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_cli_gpu.py -q -k graph_steps_equal --timeout 200 --timeout-method thread > gpurun_out/r4f/graph.log 2>&1; tail -40 gpurun_out/r4f/graph.log | cut -c1-250
