#!/bin/bash
# Rebuild only norm.hip with extra flags and link it with the in-tree objects into variants/<name>/
# (GroupNorm A/B experiments; run with MVAE_HIP_LIB=variants/<name>/libmvae_hip.so).
# usage: tools/build_norm_variant.sh <name> [extra hipcc flags...]
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/variants/$NAME
mkdir -p "$OUT"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fno-slp-vectorize --offload-arch=gfx950 -w "$@" \
  -c "$ROOT/medvae_disentangled_multimodal_amd/csrc/norm.hip" -o "$OUT/norm.hip.o"
objs=$(ls "$ROOT"/build/*.o | grep -v '/norm.hip.o$')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs "$OUT/norm.hip.o" -o "$OUT/libmvae_hip.so"
rm -f "$OUT/norm.hip.o"
echo "built $OUT/libmvae_hip.so"
