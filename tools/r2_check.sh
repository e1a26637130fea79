#!/bin/bash
# GPU validation pass: GPU tests, smoke, benches of c4 / c2 / c3 (each under its own time limit; stop at the first failure).
TAG=${1:-r2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
for c in c4 c2 c3; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --detail > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err || exit $?
  cat gpurun_out/${TAG}_bench_$c.json | cut -c1-400
done
