#!/bin/bash
# one model's step profile + bench on the same box: prof_one.sh <tag> <Model> <batch>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
export PCA_TUNE_CACHE=/tmp/tune_prof.json
tag=$1; m=$2; b=$3
timeout -k 10 200 python bench.py --model $m --batch $b --steps 5 --warmup 3 > /dev/null 2>&1 || exit 1
BENCH_ARGS="--model $m" bash tools/gpu/prof_bench.sh ${tag}_$m $b > /dev/null 2>&1 || exit 1
timeout -k 10 200 python bench.py --model $m --batch $b --steps 30 --warmup 10 2>/dev/null | tail -1 > gpurun_out/prof/${tag}_${m}_b${b}_bench.json || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/prof/${tag}_${m}_b${b}_bench.json')); print('$m b$b %.3f ms' % d['ms_per_step'])"
