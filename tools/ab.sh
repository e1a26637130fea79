# A/B of kernel variants (variants/<name>/libmvae_hip.so) on the per-shape conv bench, interleaved rounds
set -e
mkdir -p gpurun_out
for r in 1 2; do
for v in "$@"; do
  echo "== $v" >> gpurun_out/ab.log
  MVAE_HIP_LIB=variants/$v/libmvae_hip.so timeout -k 10 200 python tools/conv_bench.py >> gpurun_out/ab.log 2>&1
done
done
