#!/bin/bash
# HBM traffic of the GEMM kernel family over one training step (config $1, default c4):
# two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE), kernel-trace only, then
# tools/pmc_traffic.py applies the gfx950 correction (FETCH_SIZE x2) and writes per-launch bytes.
set -e
CFG=${1:-c4}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-include-regex gemm3x -d gpurun_out/traffic_${CFG}_$C -o run \
    --output-format csv -- python bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timing \
    > gpurun_out/traffic_${CFG}_$C.log 2>&1
done
python3 tools/pmc_traffic.py $CFG ${2:-r02}
