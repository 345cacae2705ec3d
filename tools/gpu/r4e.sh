#!/bin/bash
# A/B: hx forward interleave, depthwise BN fusion (MobileNetV2 / EfficientNet-B0), Winograd stages
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4e
for v in 1 0 1 0; do
  PCA_HX_ILV=$v timeout -k 10 300 python bench.py --batch 1024 --steps 20 --warmup 5 > gpurun_out/r4e/ilv$v.json 2>/dev/null || exit 1
  echo "ilv=$v $(cat gpurun_out/r4e/ilv$v.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"])')"
done
for m in MobileNetV2:1024 EfficientNetB0:128 EfficientNetB0:1024; do
  model=${m%%:*}; b=${m##*:}
  for v in 1 0; do
    PCA_DW_IN_FUSE=$v timeout -k 10 300 python bench.py --model $model --batch $b --steps 20 --warmup 5 > gpurun_out/r4e/${model}_${b}_${v}.json 2>gpurun_out/r4e/${model}_${b}_${v}.err || { tail -5 gpurun_out/r4e/${model}_${b}_${v}.err; exit 1; }
    echo "$model bs$b dwfuse=$v $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d["value"])' gpurun_out/r4e/${model}_${b}_${v}.json)"
  done
done
timeout -k 10 300 python -u tools/winograd_ab.py --batch 1024 > gpurun_out/r4e/winograd.jsonl 2>&1; tail -4 gpurun_out/r4e/winograd.jsonl
