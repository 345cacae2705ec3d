#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/wp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "weight_prep or zoo_matches or resnet18 or graph or mobilenet" > gpurun_out/wp/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/wp/pytest.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/prof_bench.sh wp 1024 128
