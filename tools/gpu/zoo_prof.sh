#!/bin/bash
# kernel-family summaries of the zoo models' bench steps (non-native kernels flagged)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for m in ${MODELS:-ShuffleNetG2 DPN26 EfficientNetB0}; do
  BENCH_ARGS="--model $m" bash tools/gpu/prof_bench.sh $m ${BATCH:-128} || exit 1
  f=gpurun_out/prof/${m}_b${BATCH:-128}_timeline.txt
  echo "== $m"; sed -n '1,40p' $f | grep -E "kernels:|at::native|Cijk|elementwise|reduce_kernel|copyBuffer|fill" || true
done
