#!/bin/bash
# HBM traffic of one kernel family over one training step (config $1, default c4; output tag $2; family $3:
# gemm3x (default) or gn_ = the GroupNorm chains): two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE),
# kernel-trace only, then tools/pmc_traffic.py applies the gfx950 correction (FETCH_SIZE x2) and writes per-launch
# and per-step bytes.
set -e
CFG=${1:-c4}; TAG=${2:-r03}; FAM=${3:-gemm3x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-include-regex "$FAM" -d gpurun_out/traffic_${CFG}_${FAM}_$C -o run \
    --output-format csv -- python bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timing \
    --no-parity > gpurun_out/traffic_${CFG}_${FAM}_$C.log 2>&1
done
python3 tools/pmc_traffic.py $CFG $TAG $FAM
