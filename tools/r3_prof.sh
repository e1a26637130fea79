#!/bin/bash
# rocprofv3 kernel summary of one config's bench run: tools/r3_prof.sh <tag> <config> [steps]
TAG=${1:-p}; CFG=${2:-c3}; STEPS=${3:-3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof_$CFG -o run --output-format csv -- python3 bench.py --config $CFG --steps $STEPS --warmup 1 --no-cpu-baseline --no-kernel-timing > gpurun_out/$TAG/prof_$CFG.log 2>&1 || exit $?
f=$(find gpurun_out/$TAG/prof_$CFG -name "*kernel_stats.csv" | head -1); head -30 "$f" | cut -d, -f1-4 | cut -c1-160
