#!/bin/bash
# Round-over-round, one box: ab_r3 (round-3 final build, rebuilt in a worktree) vs this tree.
# ResNet-18 bs1024 / bs128 x2, DPN26 / RegNetX_200MF / RegNetY_400MF / MobileNetV2 bs256.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r4x
mkdir -p $O
ms() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"])' $1; }
for rep in 1 2; do
  for b in 1024 128; do
    for v in ab_r3 .; do
      n=$(basename $(cd $v && pwd))
      (cd $v && timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10) > $O/${n}_${b}_$rep.json 2>$O/err.log || { tail -5 $O/err.log; exit 1; }
      echo "rep$rep ResNet18 bs$b $n $(ms $O/${n}_${b}_$rep.json)"
    done
  done
done
for m in DPN26 RegNetX_200MF RegNetY_400MF MobileNetV2; do
  for v in ab_r3 .; do
    n=$(basename $(cd $v && pwd))
    (cd $v && timeout -k 10 300 python bench.py --model $m --batch 256 --steps 20 --warmup 5) > $O/${n}_$m.json 2>$O/err.log || { tail -5 $O/err.log; exit 1; }
    echo "$m bs256 $n $(ms $O/${n}_$m.json)"
  done
done
exit 0
