#!/bin/bash
# same-box A/B: current default (halo wgrad DMA interleave on) vs round 3 vs two build-time variants
# (hx forward DMA after fragment reads; igemm DMA after fragment reads), + numerics of the variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r4r
mkdir -p $O
ROOT=$PWD
for v in variant_hx variant_sp; do
  rm -rf $v/tests && cp -r tests $v/tests   # (the variant trees ship without tests)
  (cd $v && timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -q -k "conv or halo" --timeout 300 --timeout-method thread -p no:cacheprovider) > $O/pytest_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc"; tail -1 $O/pytest_$v.log; grep -E "^FAILED" $O/pytest_$v.log | head -5
  [ $rc -ne 0 ] && exit 1
done
ms() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"])' $1; }
for rep in 1 2; do
  for b in 1024 128; do
    (cd baseline_r3 && timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10) > $O/r3_${b}_$rep.json 2>$O/r3.err || exit $?
    timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10 > $O/cur_${b}_$rep.json 2>$O/cur.err || exit $?
    (cd variant_hx && timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10) > $O/hx_${b}_$rep.json 2>$O/hx.err || { tail -5 $O/hx.err; exit 1; }
    (cd variant_sp && timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10) > $O/sp_${b}_$rep.json 2>$O/sp.err || { tail -5 $O/sp.err; exit 1; }
    echo "rep$rep bs$b r3 $(ms $O/r3_${b}_$rep.json) cur $(ms $O/cur_${b}_$rep.json) hx-after-read $(ms $O/hx_${b}_$rep.json) igemm-after-read $(ms $O/sp_${b}_$rep.json)"
  done
done
exit 0
