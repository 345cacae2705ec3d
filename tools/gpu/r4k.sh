#!/bin/bash
# graph-vs-eager with pre-linked zero pilots; shift kernel test; full GPU suite; tune logs; traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
PRELINK=1 timeout -k 10 200 python -u tools/diag/graph_eager.py > $O/ge_prelink.log 2>&1 || exit $?
echo "prelink:"; grep step $O/ge_prelink.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -gt 1 ] && exit $rc
for b in 1024 128; do
  PCA_TUNE_LOG=1 timeout -k 10 300 python bench.py --batch $b --steps 20 --warmup 5 \
    > $O/tune_b$b.json 2> $O/tune_b$b.log || exit 1
  cat $O/tune_b$b.json
done
bash tools/gpu/prof_bench.sh r4k 1024 128 || exit 1
exit 0
