#!/bin/bash
# Shift-kernel identity test, graph-vs-eager with/without shift, same-box A/B against round 3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_bn_shift_gpu.py -x -q --timeout 120 --timeout-method thread > $O/shift.log 2>&1; rc=$?
tail -5 $O/shift.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for s in 1 0; do
  PCA_BN_SHIFT=$s timeout -k 10 200 python -u tools/diag/graph_eager.py > $O/ge$s.log 2>&1 || exit $?
  echo "shift=$s"; grep step $O/ge$s.log
done
ms() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"])' $1; }
for rep in 1 2; do
  for b in 1024 128; do
    (cd baseline_r3 && timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10) > $O/r3_${b}_$rep.json 2>$O/r3.err || exit $?
    timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10 > $O/cur_${b}_$rep.json 2>$O/cur.err || exit $?
    PCA_BN_SHIFT=0 timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10 > $O/ns_${b}_$rep.json 2>$O/ns.err || exit $?
    echo "rep$rep bs$b r3 $(ms $O/r3_${b}_$rep.json) cur $(ms $O/cur_${b}_$rep.json) noshift $(ms $O/ns_${b}_$rep.json)"
  done
done
