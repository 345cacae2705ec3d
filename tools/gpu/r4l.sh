#!/bin/bash
# zero-pilot training-step diag; full GPU suite (MIOpen off in references); same-box A/B vs round 3; traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 200 python -u tools/diag/pilot_zero.py > $O/pz.log 2>&1 || exit $?
grep -v Warn $O/pz.log | tail -2
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -gt 1 ] && exit $rc
ms() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"])' $1; }
for rep in 1 2; do
  for b in 1024 128; do
    (cd baseline_r3 && timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10) > $O/r3_${b}_$rep.json 2>$O/r3.err || exit $?
    timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10 > $O/cur_${b}_$rep.json 2>$O/cur.err || exit $?
    PCA_WGRAD_STREAM=1 timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10 > $O/ws_${b}_$rep.json 2>$O/ws.err || exit $?
    echo "rep$rep bs$b r3 $(ms $O/r3_${b}_$rep.json) cur $(ms $O/cur_${b}_$rep.json) wgrad-stream $(ms $O/ws_${b}_$rep.json)"
  done
done
bash tools/gpu/prof_bench.sh r4l 1024 128 || exit 1
exit 0
