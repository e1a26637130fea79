#!/bin/bash
# rocprofv3 kernel-trace stats of the bench (warmup 0, no live timing): tools/prof_run.sh <tag> <config> [steps]
TAG=$1; CFG=$2; STEPS=${3:-3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_${CFG}_prof -o run --output-format csv -- python3 bench.py --config $CFG --steps $STEPS --warmup 0 --no-cpu-baseline --no-kernel-timing > gpurun_out/${TAG}_${CFG}_prof.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_${CFG}_prof.log | cut -c1-200
