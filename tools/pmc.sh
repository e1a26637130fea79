#!/bin/bash
# Collect PMC counter sets (one rocprofv3 pass each, kernel-trace only, no tracing domains) for one
# conv pass of tools/one_conv.py.   usage: tools/pmc.sh <shape> <pass> <outprefix>
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SHAPE=$1; PASS=$2; OUT=$3
SETS=(
 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA"
 "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD"
 "TA_TA_BUSY TD_TD_BUSY TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES"
 "TCC_HIT TCC_MISS TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM"
 "TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_TOTAL_CACHE_ACCESSES TCP_CACHE_MISS"
)
i=0
for P in "${SETS[@]}"; do
  timeout -k 10 150 rocprofv3 --pmc $P --kernel-include-regex gemm3x -d gpurun_out/${OUT}_$i -o run --output-format csv -- python tools/one_conv.py --shape $SHAPE --pass_ $PASS --reps 3 > gpurun_out/${OUT}_$i.log 2>&1
  i=$((i+1))
done
