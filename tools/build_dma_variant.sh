#!/bin/bash
# variants/<name>/libmvae_hip.so = the current objects with gemm_dma.hip rebuilt under extra flags
set -e
NAME=$1; shift
cd "$(dirname "$0")/.."
mkdir -p variants/$NAME
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fno-slp-vectorize --offload-arch=gfx950 -w "$@" -c medvae_disentangled_multimodal_amd/csrc/gemm_dma.hip -o variants/$NAME/gemm_dma.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $(ls build/*.o | grep -v gemm_dma) variants/$NAME/gemm_dma.o -o variants/$NAME/libmvae_hip.so
rm variants/$NAME/gemm_dma.o
echo built variants/$NAME
