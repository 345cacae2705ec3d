#!/bin/bash
# PMC counter passes on one conv kernel (tools/conv_one.py args forwarded). Writes CSVs under
# gpurun_out/pmc/<tag>_<pass>/. Each pass is its own rocprofv3 run (counters + kernel trace only).
# usage: tools/pmc_conv.sh <tag> [conv_one.py args...]
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc/${tag}_p$i -o run -- python tools/conv_one.py "$@" > gpurun_out/pmc/${tag}_p$i.log 2>&1
done
