#!/bin/bash
# Round-4 first GPU pass: round-end rehearsal (GPU suite, smoke, bench), autotune trial log of the
# bs1024 / bs128 steps, and kernel traces of both.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4a
bash tools/gpu/round_end.sh || exit $?
for b in 1024 128; do
  PCA_TUNE_LOG=1 timeout -k 10 300 python bench.py --batch $b --steps 10 --warmup 5 \
    > gpurun_out/r4a/tune_b$b.json 2> gpurun_out/r4a/tune_b$b.log || exit 1
  grep -c "\[tune\]" gpurun_out/r4a/tune_b$b.log
done
bash tools/gpu/prof_bench.sh r4a 1024 128
