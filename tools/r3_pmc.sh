#!/bin/bash
# PMC passes (kernel-trace only, one counter set per rocprofv3 run) of single conv passes, 3xBF16 vs bf16:
#   tools/r3_pmc.sh <tag> "<shape> ..." "<pass> ..." "<precision> ..."
TAG=${1:-pmc}; SHAPES=${2:-3}; PASSES=${3:-fwd}; PRECS=${4:-"32 bf16-mixed"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
SETS=(
 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA"
 "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_SCA SQ_INSTS_SALU"
)
for S in $SHAPES; do for P in $PASSES; do for PR in $PRECS; do
  i=0
  for C in "${SETS[@]}"; do
    O=gpurun_out/$TAG/s${S}_${P}_${PR}_$i
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex gemm3x -d $O -o run --output-format csv -- python3 tools/one_conv.py --shape $S --pass_ $P --reps 3 --precision $PR > $O.log 2>&1 || exit $?
    i=$((i+1))
  done
  echo "== shape $S $P $PR"; python3 tools/pmc_summary.py "gpurun_out/$TAG/s${S}_${P}_${PR}_*/**/*counter_collection.csv"
done; done; done
