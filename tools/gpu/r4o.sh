#!/bin/bash
# dual-BN aux2 through LDS / registers: dgrad numerics, same-box A/B on ResNet-18 vs round 3, trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_production_gpu.py -q -k "dual or dgrad or ResNet18 or every_tile" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^E " $O/pytest.log | head -20
[ $rc -gt 1 ] && exit $rc
ms() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"])' $1; }
for rep in 1 2; do
  for b in 1024 128; do
    (cd baseline_r3 && timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10) > $O/r3_${b}_$rep.json 2>$O/r3.err || exit $?
    timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10 > $O/cur_${b}_$rep.json 2>$O/cur.err || exit $?
    echo "rep$rep bs$b r3 $(ms $O/r3_${b}_$rep.json) cur $(ms $O/cur_${b}_$rep.json)"
  done
done
bash tools/gpu/prof_bench.sh r4o 1024 128 || exit 1
exit 0
