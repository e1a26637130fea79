#!/bin/bash
# GPU test suite (+ optional benches): tools/gpu_suite.sh <tag> [config ...]
TAG=${1:-t}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/${TAG}_pytest.log | head -20; tail -2 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for c in "$@"; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --detail > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err || exit $?
  cut -c1-300 gpurun_out/${TAG}_bench_$c.json
done
