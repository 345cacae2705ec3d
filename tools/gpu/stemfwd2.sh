#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sf2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "conv_fwd_dgrad or resnet18 or zoo_matches" > gpurun_out/sf2/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/sf2/pytest.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/prof_bench.sh sf2 1024 128
