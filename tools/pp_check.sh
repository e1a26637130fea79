#!/bin/bash
# Ping-pong GEMM variant: kernel tests against float64 torch, then per-shape and c4 A/B vs the base library.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V=${1:-pp}
MVAE_HIP_LIB=variants/$V/libmvae_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${V}_tests.log 2>&1 || { tail -30 gpurun_out/${V}_tests.log; exit 1; }
tail -2 gpurun_out/${V}_tests.log
rm -f gpurun_out/ab.log
timeout -k 10 600 bash tools/ab.sh base $V || exit $?
cat gpurun_out/ab.log
CFG=c4 timeout -k 10 500 bash tools/ab_lib.sh c4ab base $V
