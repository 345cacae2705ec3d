#!/bin/bash
# Mobile nets after the igemm dgrad epilogue change: MobileNetV2 bs1024, EfficientNet-B0 bs1024 / bs128.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r4w
mkdir -p $O
for mb in MobileNetV2:1024 EfficientNetB0:1024 EfficientNetB0:128; do
  m=${mb%%:*}; b=${mb##*:}
  timeout -k 10 400 python bench.py --model $m --batch $b --steps 30 --warmup 10 > $O/${m}_$b.json 2> $O/${m}_$b.err || { tail -5 $O/${m}_$b.err; exit 1; }
  cat $O/${m}_$b.json
done
exit 0
