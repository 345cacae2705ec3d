#!/bin/bash
# round-3d check: full GPU suite + benches (tools/gpu/round_check.sh), then ResNet-18 step profiles
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu/round_check.sh || exit 1
grep -q "pytest rc=0" gpurun_out/rc/pytest.log 2>/dev/null; tail -3 gpurun_out/rc/pytest.log | grep -q failed && exit 1
export PCA_TUNE_CACHE=/tmp/tune_prof.json
for b in 1024 128; do
  timeout -k 10 200 python bench.py --batch $b --steps 5 --warmup 3 > /dev/null 2>&1 || exit 1
done
bash tools/gpu/prof_bench.sh r3d 1024 128
