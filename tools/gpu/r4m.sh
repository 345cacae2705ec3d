#!/bin/bash
# real-RCCL world-1 graph DDP test; mobile-net traces (stock at:: kernels?); DPN26 / RegNet same-box vs round 3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ddp_gpu.py -q --timeout 240 --timeout-method thread > $O/ddp.log 2>&1
rc=$?; echo "ddp rc=$rc"; tail -2 $O/ddp.log; grep -E "^FAILED|^E " $O/ddp.log | head -10
[ $rc -gt 1 ] && exit $rc
ms() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"])' $1; }
for m in DPN26 RegNetX_200MF RegNetY_400MF; do
  (cd baseline_r3 && timeout -k 10 300 python bench.py --model $m --batch 256 --steps 20 --warmup 5) > $O/r3_$m.json 2>$O/r3.err || exit $?
  timeout -k 10 300 python bench.py --model $m --batch 256 --steps 20 --warmup 5 > $O/cur_$m.json 2>$O/cur.err || exit $?
  echo "$m bs256 r3 $(ms $O/r3_$m.json) cur $(ms $O/cur_$m.json)"
done
BENCH_ARGS="--model MobileNetV2" bash tools/gpu/prof_bench.sh mnv2_r4m 1024 || exit 1
BENCH_ARGS="--model EfficientNetB0" bash tools/gpu/prof_bench.sh effb0_r4m 128 1024 || exit 1
exit 0
