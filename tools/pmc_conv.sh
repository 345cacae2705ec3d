#!/bin/bash
# PMC counter passes on one conv kernel (tools/conv_one.py args forwarded). Writes CSVs under
# gpurun_out/pmc/<tag>_p<i>/. Each pass is its own rocprofv3 run (counters + kernel trace only).
# usage: tools/pmc_conv.sh <tag> [conv_one.py args...]   (PMC_EXTRA=1 adds two more passes)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
SETS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
      "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum")
if [ -n "$PMC_EXTRA" ]; then
  SETS+=("SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_INST_CYCLES_VMEM_RD"
         "TA_TA_BUSY_sum TA_BUFFER_READ_LDS_WAVEFRONTS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_LATENCY_sum")
fi
mkdir -p gpurun_out/pmc
i=0
for P in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc/${tag}_p$i -o run -- python tools/conv_one.py "$@" > gpurun_out/pmc/${tag}_p$i.log 2>&1
done
