#!/bin/bash
# interleaved A/B of DMA main-loop variants on tools/dma_exp.py: tools/dma_ab.sh <tag> <variant> ... ("default" = in-tree lib)
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = default ]; then L=""; else L="MVAE_HIP_LIB=variants/$v/libmvae_hip.so"; fi
    env $L timeout -k 10 120 python3 tools/dma_exp.py >> gpurun_out/$TAG/ab.log 2>&1 || exit $?
  done
done
cat gpurun_out/$TAG/ab.log | grep -v amdgpu.ids
