#!/bin/bash
# igemm epilogue: operands of a store-loop chunk loaded together (one memory round trip per chunk);
# BN-sum block flush by wave butterfly + one LDS row per wave.
# Numerics on this tree (chunk 2), then A/B: ab_head (previous commit) vs this tree vs ab_eu1
# (chunk 1), bench bs1024 / bs128, and kernel traces of both variants at bs1024.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r4u
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_ops_gpu.py tests/test_kernels_gpu.py tests/test_production_gpu.py -q -k "dual or dgrad or every_tile or fusion or ResNet18 or split" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; grep -E "^FAILED" $O/pytest.log | head -10
[ $rc -ne 0 ] && exit 1
ms() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"])' $1; }
for rep in 1 2; do
  for b in 1024 128; do
    for v in ab_head . ab_eu1; do
      n=$(basename $(cd $v && pwd))
      (cd $v && timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10) > $O/${n}_${b}_$rep.json 2>$O/err.log || { tail -5 $O/err.log; exit 1; }
      echo "rep$rep bs$b $n $(ms $O/${n}_${b}_$rep.json)"
    done
  done
done
for v in . ab_eu1; do
  n=$(basename $(cd $v && pwd)); d=$PWD/$O/prof_$n
  (cd $v && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --steps 10 --warmup 5 --batch 1024 > $d.log 2>&1) || { tail -20 $d.log; exit 1; }
  f=$(ls $d/*kernel_trace.csv $d/*/*kernel_trace.csv 2>/dev/null | head -1)
  python3 tools/step_timeline.py "$f" > $O/timeline_$n.txt || exit 1
  head -2 $O/timeline_$n.txt
done
exit 0
