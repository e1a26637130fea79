#!/bin/bash
# MFMA-structure ceilings (micro) + PMC wait/issue breakdown of the c4 8x8x2048 conv GEMMs (fwd / dgrad / wgrad).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./tools/micro/mfma_shape > gpurun_out/micro_shape.txt 2>&1 || exit $?
timeout -k 10 120 ./tools/micro/mfma_peak > gpurun_out/micro_peak.txt 2>&1 || exit $?
cat gpurun_out/micro_shape.txt gpurun_out/micro_peak.txt
timeout -k 10 900 bash tools/pmc_passes.sh 3 pmc8
