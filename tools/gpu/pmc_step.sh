#!/bin/bash
# PMC counters of one eager bench step per batch size: each counter set is its own
# rocprofv3 run (counters + kernel trace only), summarised by tools/pmc_step.py; the raw CSVs
# are deleted after the summary (gpurun copies back at most 64 MiB).
# usage: bash tools/gpu/pmc_step.sh <tag> <batch>...   (extra bench args via BENCH_ARGS)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
tag=$1; shift
SETS=("SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
      "FETCH_SIZE"
      "WRITE_SIZE")
mkdir -p gpurun_out/pmc_step
for b in "$@"; do
  # tune once without the profiler (rocprof serialisation distorts the autotuner's timings),
  # then every pass replays those choices
  export PCA_TUNE_CACHE=/tmp/pmc_tune_${tag}_b$b.json
  rm -f $PCA_TUNE_CACHE
  timeout -k 10 240 python3 bench.py --steps 3 --warmup 3 --batch $b $BENCH_ARGS > gpurun_out/pmc_step/${tag}_b${b}_tune.log 2>&1 \
    || { echo "FAILED tune b=$b"; tail -20 gpurun_out/pmc_step/${tag}_b${b}_tune.log; exit 1; }
  cp $PCA_TUNE_CACHE gpurun_out/pmc_step/${tag}_b${b}_tune.json
  i=0
  for P in "${SETS[@]}"; do
    i=$((i+1))
    d=/tmp/pmc_step/${tag}_b${b}_p$i
    timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $d -o run -- \
      python3 bench.py --graph 0 --steps 3 --warmup 3 --batch $b $BENCH_ARGS > gpurun_out/pmc_step/${tag}_b${b}_p$i.log 2>&1 \
      || { echo "FAILED b=$b pass $i"; tail -20 gpurun_out/pmc_step/${tag}_b${b}_p$i.log; exit 1; }
    echo "b=$b pass $i done"
  done
  f=$(ls /tmp/pmc_step/${tag}_b${b}_p1/*counter_collection.csv /tmp/pmc_step/${tag}_b${b}_p1/*/*counter_collection.csv 2>/dev/null | head -1)
  head -3 "$f" > gpurun_out/pmc_step/${tag}_b${b}_counter_head.csv
  python3 tools/pmc_step.py /tmp/pmc_step/${tag}_b${b}_p* --top 60 > gpurun_out/pmc_step/${tag}_b${b}.txt || exit 1
  rm -rf /tmp/pmc_step/${tag}_b${b}_p*
  head -30 gpurun_out/pmc_step/${tag}_b${b}.txt
done
