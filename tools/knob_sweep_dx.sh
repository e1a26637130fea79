#!/bin/bash
# The unwritten-GroupNorm-dx test (NaN-poisoned buffer) under each opt-in / opt-out conv-backward knob: a knob that routes
# conv1 to a kernel reading the fp32 dy shows up as a failure (tools/ script, run on the GPU box through gpurun).
set -e
mkdir -p gpurun_out/r06k
for knob in MVAE_NO_WINOGRAD_WGRAD=1 MVAE_BWD_OVERLAP=0 MVAE_NO_WGRAD_P2=1 MVAE_NO_DIRECT32=1 MVAE_NO_WINOGRAD_DY2=1 MVAE_NO_WINOGRAD_KEEP_V=1 MVAE_NO_BF16_DMA=1; do
  echo "== $knob" >> gpurun_out/r06k/knobs.log
  env $knob timeout -k 10 300 python -u -m pytest tests/test_gpu_gn_pack.py -k unwritten -q --timeout 120 --timeout-method thread >> gpurun_out/r06k/knobs.log 2>&1
done
tail -3 gpurun_out/r06k/knobs.log
