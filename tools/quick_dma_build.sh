#!/bin/bash
# Rebuild only the LDS-DMA GEMM translation unit and relink (valid while gemm_core.h edits touch PREC 4 code only;
# a change to shared kernel code needs the full `make`).
set -e
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fno-slp-vectorize --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-variable -c medvae_disentangled_multimodal_amd/csrc/gemm_dma.hip -o build/gemm_dma.hip.o
touch build/*.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build/*.o -o medvae_disentangled_multimodal_amd/libmvae_hip.so
echo relinked
