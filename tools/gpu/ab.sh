#!/bin/bash
# Same-box A/B runner (one script for every comparison of the rounds' notes).
#
#   bash tools/gpu/ab.sh [-t '<pytest args, e.g. tests/x.py -k "a or b">'] [-r REPS] [-b "BATCHES"] [-m "Model batch"]... ARM ARM...
#
# An ARM is a source tree holding bench.py + a built pytorch_cifar_amd/, optionally followed by
# "|" and environment settings:  "."  "ab/base"  ".|PCA_GROUP_DENSE=0"  ".|PCA_S2C_ADDEND=0".
# (A base tree for a code change: git archive HEAD pytorch_cifar_amd bench.py __graft_entry__.py
#  | tar -x -C ab/base, build it in place, and take ./ab out of .gpurunignore for the call.)
# Benches: the ResNet-18 headline step at each of -b BATCHES (default "1024 128"), or each
# -m "Model batch". Each arm tunes once into its own cache, then REPS (default 3) interleaved
# repetitions print "<arm> <config> <ms/step>". -t runs that pytest selection first (in ".").
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS=""; REPS=3; BATCHES="1024 128"; MODELS=()
while getopts "t:r:b:m:" o; do
  case $o in
    t) TESTS=$OPTARG ;;
    r) REPS=$OPTARG ;;
    b) BATCHES=$OPTARG ;;
    m) MODELS+=("$OPTARG") ;;
    *) exit 2 ;;
  esac
done
shift $((OPTIND - 1))
[ $# -ge 2 ] || { echo "need at least two arms"; exit 2; }
ARMS=("$@")
if [ -n "$TESTS" ]; then
  # (eval: quotes inside the -t string group a -k expression)
  eval "timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS" \
    > gpurun_out/ab_tests.log 2>&1 || { tail -40 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi
CFGS=()
if [ ${#MODELS[@]} -gt 0 ]; then CFGS=("${MODELS[@]}"); else for b in $BATCHES; do CFGS+=("ResNet18 $b"); done; fi
run() {   # run <arm-index> <arm> <model> <batch> <steps> <warmup>
  local dir=${2%%|*} env=""
  [[ $2 == *"|"* ]] && env=${2#*|}
  env $env PCA_TUNE_CACHE=/tmp/tune_ab_$1.json timeout -k 10 300 \
    python $dir/bench.py --model $3 --batch $4 --steps $5 --warmup $6 2>/dev/null
}
i=0
for arm in "${ARMS[@]}"; do   # tuning pass per arm and config
  for c in "${CFGS[@]}"; do
    set -- $c
    run $i "$arm" $1 $2 5 3 > /dev/null || { echo "arm [$arm] $c failed"; exit 1; }
  done
  i=$((i + 1))
done
for rep in $(seq $REPS); do
  i=0
  for arm in "${ARMS[@]}"; do
    for c in "${CFGS[@]}"; do
      set -- $c
      run $i "$arm" $1 $2 30 10 | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('[$arm] $1 b$2', d['ms_per_step'])" || exit 1
    done
    i=$((i + 1))
  done
done
