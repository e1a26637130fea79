#!/bin/bash
# Collect PMC counter sets (one rocprofv3 pass each, no tracing domains) for one conv pass.
# usage: tools/pmc.sh <shape> <pass> <outprefix>
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SHAPE=$1; PASS=$2; OUT=$3
SETS=(
 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
 "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"
 "TCC_HIT_sum TCC_MISS_sum"
 "FETCH_SIZE"
 "WRITE_SIZE"
)
i=0
for P in "${SETS[@]}"; do
  timeout -k 10 150 rocprofv3 --pmc $P --kernel-include-regex gemm3x -d gpurun_out/${OUT}_$i -o run --output-format csv -- python tools/one_conv.py --shape $SHAPE --pass_ $PASS --reps 3 > gpurun_out/${OUT}_$i.log 2>&1
  i=$((i+1))
done
