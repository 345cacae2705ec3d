#!/bin/bash
# PMC counters of one eager bench step per batch size: each counter set is its own
# rocprofv3 run (counters + kernel trace only), summarised by tools/pmc_step.py.
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
  i=0
  for P in "${SETS[@]}"; do
    i=$((i+1))
    d=gpurun_out/pmc_step/${tag}_b${b}_p$i
    timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $d -o run -- \
      python3 bench.py --graph 0 --steps 3 --warmup 3 --batch $b $BENCH_ARGS > $d.log 2>&1 \
      || { echo "FAILED b=$b pass $i"; tail -20 $d.log; exit 1; }
    echo "b=$b pass $i done"
  done
  python3 tools/pmc_step.py gpurun_out/pmc_step/${tag}_b${b}_p* --top 40 > gpurun_out/pmc_step/${tag}_b${b}.txt || exit 1
  head -25 gpurun_out/pmc_step/${tag}_b${b}.txt
done
