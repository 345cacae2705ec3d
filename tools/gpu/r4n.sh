#!/bin/bash
# no-activation BN backward fusion: numerics (production + ops + ddp tests), same-box A/B on the mobile nets.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_production_gpu.py tests/test_ops_gpu.py tests/test_ddp_gpu.py -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^E " $O/pytest.log | head -20
[ $rc -gt 1 ] && exit $rc
ms() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"])' $1; }
for mb in MobileNetV2:1024 EfficientNetB0:128 EfficientNetB0:1024; do
  m=${mb%%:*}; b=${mb##*:}
  for v in 1 0 1 0; do
    PCA_FUSE_BN_NOACT=$v timeout -k 10 300 python bench.py --model $m --batch $b --steps 20 --warmup 5 > $O/${m}_${b}_$v.json 2>$O/err.log || { tail -5 $O/err.log; exit 1; }
    echo "$m bs$b noact-fuse=$v $(ms $O/${m}_${b}_$v.json)"
  done
done
BENCH_ARGS="--model EfficientNetB0" bash tools/gpu/prof_bench.sh effb0_r4n 128 || exit 1
exit 0
