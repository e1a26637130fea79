#!/bin/bash
# Round-3 PMC evidence: counter passes of the 8x8x2048 conv (fwd / dgrad / wgrad, 3xBF16 and bf16-mixed) and the
# per-step HBM traffic of the GroupNorm family (c4, c3).   tools/r3_pmc_evidence.sh <tag>
TAG=${1:-pmcev}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
bash tools/r3_pmc.sh $TAG 3 "fwd dgrad wgrad" "32 bf16-mixed" > gpurun_out/$TAG/pmc_conv.txt 2>&1 || exit $?
bash tools/pmc_traffic.sh c4 r03 gn_ > gpurun_out/$TAG/gn_c4.txt 2>&1 || exit $?
bash tools/pmc_traffic.sh c3 r03 gn_ > gpurun_out/$TAG/gn_c3.txt 2>&1 || exit $?
mkdir -p gpurun_out/$TAG/profiles && cp profiles/r03_c4_gn_traffic.json profiles/r03_c3_gn_traffic.json gpurun_out/$TAG/profiles/
tail -3 gpurun_out/$TAG/gn_c4.txt gpurun_out/$TAG/gn_c3.txt
