#!/bin/bash
# rocprofv3 kernel traces of the hipGraph bench step at the given per-GPU batches.
# usage: bash tools/gpu/prof_bench.sh <tag> <batch>... (extra bench args via BENCH_ARGS)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/prof
for b in "$@"; do
  d=gpurun_out/prof/${tag}_b$b
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
    python3 bench.py --steps 10 --warmup 5 --batch $b $BENCH_ARGS > $d.log 2>&1 || { echo "FAILED b=$b"; tail -20 $d.log; exit 1; }
  tail -1 $d.log
  f=$(ls $d/*kernel_trace.csv $d/*/*kernel_trace.csv 2>/dev/null | head -1)
  python3 tools/step_timeline.py "$f" > gpurun_out/prof/${tag}_b${b}_timeline.txt || exit 1
  head -2 gpurun_out/prof/${tag}_b${b}_timeline.txt
done
