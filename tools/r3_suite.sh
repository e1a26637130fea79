#!/bin/bash
# Round-3 GPU check: the -m gpu suite, then the driver's default bench command (c4 + c2/c3/c5 + parity block).
#   tools/r3_suite.sh <tag> [bench]
TAG=${1:-t}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/$TAG/pytest.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
if [ "$2" = bench ]; then
  timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
  cut -c1-400 gpurun_out/$TAG/bench.json
fi
exit $rc
