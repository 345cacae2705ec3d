#!/bin/bash
# A/B bench: runs bench.py for each "NAME=ENV..." spec at each batch in $BATCHES (default 128 1024)
# usage: bash tools/gpu/ab_bench.sh "base=" "side=PCA_WGRAD_STREAM=1" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for b in ${BATCHES:-128 1024}; do
  for spec in "$@"; do
    name=${spec%%=*}; envs=${spec#*=}
    env $envs timeout -k 10 300 python3 bench.py --steps ${STEPS:-30} --warmup ${WARMUP:-10} --batch $b $BENCH_ARGS > gpurun_out/ab/${name}_b$b.json 2> gpurun_out/ab/${name}_b$b.err || { echo "FAILED $name b=$b"; tail -5 gpurun_out/ab/${name}_b$b.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab/${name}_b$b.json').read().strip().splitlines()[-1]); print('%-12s b=%-5d %8.3f ms  %10.1f img/s' % ('$name', $b, d['ms_per_step'], d['value']))"
  done
done
