#!/bin/bash
# Register-pressure fixes (shift in LDS / padding correction / stem waves) A/B vs round 3,
# zero-pilot bitwise diag, shift kernel test, then the full GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O
ms() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"])' $1; }
for rep in 1 2; do
  for b in 1024 128; do
    (cd baseline_r3 && timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10) > $O/r3_${b}_$rep.json 2>$O/r3.err || exit $?
    timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10 > $O/cur_${b}_$rep.json 2>$O/cur.err || exit $?
    echo "rep$rep bs$b r3 $(ms $O/r3_${b}_$rep.json) cur $(ms $O/cur_${b}_$rep.json)"
  done
done
timeout -k 10 200 python -u tools/diag/pilot_zero.py > $O/pz.log 2>&1 || exit $?
grep -v Warn $O/pz.log | tail -3
timeout -k 10 300 python -u -m pytest tests/test_bn_shift_gpu.py -q --timeout 120 --timeout-method thread > $O/shift.log 2>&1; rc=$?
tail -3 $O/shift.log; grep -E "^FAILED" $O/shift.log | head
[ $rc -gt 1 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
exit 0
