#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ce
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "cross_entropy or resnet18 or zoo_matches or graph or main_py or trains" > gpurun_out/ce/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/ce/pytest.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/prof_bench.sh ce 1024 128
