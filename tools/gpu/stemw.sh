#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sw
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "stem or resnet18 or zoo_matches" > gpurun_out/sw/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/sw/pytest.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/prof_bench.sh sw 1024 128
