#!/bin/bash
# halo wgrad swizzle with row bits 4-6 on the 8- / 4-wide maps: numerics + same-box A/B vs the
# previous build (variant_hx tree: the sources before this change).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r4t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -q -k "wgrad" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; grep -E "^FAILED" $O/pytest.log | head -10
[ $rc -ne 0 ] && exit 1
ms() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"])' $1; }
for rep in 1 2; do
  for b in 128 1024; do
    (cd variant_hx && timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10) > $O/prev_${b}_$rep.json 2>$O/prev.err || { tail -5 $O/prev.err; exit 1; }
    timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10 > $O/cur_${b}_$rep.json 2>$O/cur.err || exit $?
    echo "rep$rep bs$b prev $(ms $O/prev_${b}_$rep.json) cur $(ms $O/cur_${b}_$rep.json)"
  done
done
PCA_TUNE_LOG=1 timeout -k 10 300 python bench.py --batch 128 --steps 5 --warmup 2 > $O/tune128.json 2> $O/tune128.log || exit 1
bash tools/gpu/prof_bench.sh r4t 128 || exit 1
exit 0
