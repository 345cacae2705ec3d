#!/bin/bash
# Final tree check: full GPU suite, smoke(), bench at bs1024 / bs128, trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r4_final2
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for b in 1024 128; do
  timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10 > $O/bench_b$b.json 2> $O/bench_b$b.err || { tail -5 $O/bench_b$b.err; exit 1; }
  cat $O/bench_b$b.json
done
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
cat $O/bench_default.json
bash tools/gpu/prof_bench.sh r4final2 1024 128 || exit 1
exit 0
