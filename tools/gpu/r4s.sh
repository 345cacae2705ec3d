#!/bin/bash
# conflict-free BN-sum block reductions (dgrad epilogue flush, split-K reduce): numerics + A/B vs the
# previous commit's build (variant_hx tree = same sources before this change, default flags rebuilt).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r4s
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_ops_gpu.py tests/test_kernels_gpu.py tests/test_production_gpu.py -q -k "dual or dgrad or every_tile or fusion or ResNet18 or split" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; grep -E "^FAILED" $O/pytest.log | head -10
[ $rc -ne 0 ] && exit 1
ms() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"])' $1; }
for rep in 1 2; do
  for b in 1024 128; do
    (cd variant_hx && timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10) > $O/prev_${b}_$rep.json 2>$O/prev.err || { tail -5 $O/prev.err; exit 1; }
    timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10 > $O/cur_${b}_$rep.json 2>$O/cur.err || exit $?
    echo "rep$rep bs$b prev $(ms $O/prev_${b}_$rep.json) cur $(ms $O/cur_${b}_$rep.json)"
  done
done
exit 0
