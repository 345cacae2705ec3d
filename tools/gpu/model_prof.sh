#!/bin/bash
# Bench + rocprofv3 step trace of one model at the given per-GPU batches, tuning once per batch.
#   bash tools/gpu/model_prof.sh <Model> <tag> <batch>...
# Writes gpurun_out/mp/<tag>_b<batch>.json (bench line), tune_<tag>_b<batch>.json (the autotuner's
# selections, for tools/tune_table.py --merge) and prof/<tag>_b<batch>_timeline.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
model=$1; tag=$2; shift 2
mkdir -p gpurun_out/mp gpurun_out/prof
for b in "$@"; do
  tc=gpurun_out/mp/tune_${tag}_b$b.json
  PCA_TUNE_CACHE=$tc timeout -k 10 600 python3 bench.py --model $model --batch $b --steps 20 --warmup 5 \
    > gpurun_out/mp/${tag}_b$b.json 2> gpurun_out/mp/${tag}_b$b.err || { echo "bench FAILED b=$b"; tail -20 gpurun_out/mp/${tag}_b$b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/mp/${tag}_b$b.json').read().strip().splitlines()[-1]); print('$model b$b %.3f ms %.1f img/s' % (d['ms_per_step'], d['value']))" || exit 1
  d=gpurun_out/prof/${tag}_b$b
  PCA_TUNE_CACHE=$tc timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
    python3 bench.py --model $model --steps 10 --warmup 5 --batch $b > $d.log 2>&1 || { echo "prof FAILED b=$b"; tail -20 $d.log; exit 1; }
  f=$(ls $d/*kernel_trace.csv $d/*/*kernel_trace.csv 2>/dev/null | head -1)
  python3 tools/step_timeline.py "$f" > gpurun_out/prof/${tag}_b${b}_timeline.txt || exit 1
  head -2 gpurun_out/prof/${tag}_b${b}_timeline.txt
done
