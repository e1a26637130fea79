#!/bin/bash
# Build libmvae_hip.so with extra compile flags into variants/<name>/ (A/B kernel experiments:
# run with MVAE_HIP_LIB=variants/<name>/libmvae_hip.so).
# usage: tools/build_variant.sh <name> [extra hipcc flags...]
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/variants/$NAME
mkdir -p "$OUT/obj"
PKG=$ROOT/medvae_disentangled_multimodal_amd/csrc
pids=()
for f in "$PKG"/*.hip "$PKG"/errors.cpp; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fno-slp-vectorize --offload-arch=gfx950 -w "$@" -c "$f" -o "$OUT/obj/$(basename "$f").o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 "$OUT"/obj/*.o -o "$OUT/libmvae_hip.so"
rm -rf "$OUT/obj"
echo "built $OUT/libmvae_hip.so"
