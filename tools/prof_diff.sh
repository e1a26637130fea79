#!/bin/bash
# Per-step kernel summary of one config's bench run, free of set-up work: two rocprofv3 --kernel-trace --stats runs
# that differ only in the number of timed steps (S1, S2); tools/prof_diff.py divides the per-kernel differences in
# calls and time by S2 - S1, so the eager set-up step, the graph capture, the warmup and the parity block cancel.
#   tools/prof_diff.sh <tag> <config> [S1] [S2]
TAG=${1:-p}; CFG=${2:-c3}; S1=${3:-2}; S2=${4:-12}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
for S in $S1 $S2; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof_${CFG}_s$S -o run --output-format csv -- python3 bench.py --config $CFG --steps $S --warmup 1 --no-cpu-baseline --no-kernel-timing --no-parity > gpurun_out/$TAG/prof_${CFG}_s$S.log 2>&1 || exit $?
done
python3 tools/prof_diff.py gpurun_out/$TAG/prof_${CFG}_s$S1 gpurun_out/$TAG/prof_${CFG}_s$S2 $((S2 - S1)) > gpurun_out/$TAG/prof_${CFG}_per_step.txt
head -40 gpurun_out/$TAG/prof_${CFG}_per_step.txt
