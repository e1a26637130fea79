#!/bin/bash
# Round-3 profile evidence at HEAD: per-step rocprofv3 kernel tables (two runs differing in step count, so set-up,
# capture, warmup and the parity block cancel) and the PMC HBM traffic passes of the GEMM family, per config.
#   tools/r3_evidence.sh <tag> "<configs>"
TAG=${1:-ev}; CFGS=${2:-"c4 c2 c3 c5"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
for CFG in $CFGS; do
  case $CFG in c4|c5) S1=1; S2=3;; *) S1=2; S2=12;; esac
  bash tools/prof_diff.sh $TAG $CFG $S1 $S2 > /dev/null || exit $?
  head -12 gpurun_out/$TAG/prof_${CFG}_per_step.txt | cut -c1-150
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --pmc $C --kernel-include-regex gemm3x -d gpurun_out/traffic_${CFG}_$C -o run \
      --output-format csv -- python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timing --no-parity \
      > gpurun_out/$TAG/traffic_${CFG}_$C.log 2>&1 || exit $?
  done
done
