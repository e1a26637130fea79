#!/bin/bash
# PMC counter sets of the fwd / dgrad / wgrad GEMM of one conv_bench shape (LDS, VALU, MFMA, waits):
# tools/pmc_passes.sh <shape-index> <tag>; summaries in gpurun_out/<tag>_<pass>.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
SHAPE=$1; TAG=$2
mkdir -p gpurun_out
for P in fwd dgrad wgrad; do
  bash tools/pmc.sh $SHAPE $P ${TAG}_$P || exit 1
  python3 tools/pmc_summary.py "gpurun_out/${TAG}_${P}_*/*counter_collection.csv" > gpurun_out/${TAG}_$P.txt
done
paste gpurun_out/${TAG}_fwd.txt gpurun_out/${TAG}_dgrad.txt gpurun_out/${TAG}_wgrad.txt | awk '{print $1, $2, $4, $6}' | column -t
