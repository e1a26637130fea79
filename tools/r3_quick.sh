#!/bin/bash
# Quick GPU check after a kernel change: conv numerics tests, then bench lines (no CPU baseline) with --detail.
#   tools/r3_quick.sh <tag> "<pytest -k expr or files>" [config ...]
TAG=${1:-q}; TESTS=${2:-tests/test_gpu_kernels.py}; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/pytest.log
[ $rc -eq 0 ] || exit $rc
for c in "$@"; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --detail > gpurun_out/$TAG/bench_$c.json 2> gpurun_out/$TAG/bench_$c.err || exit $?
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/$TAG/bench_$c.json')); r=d['roofline']
print('$c', d['value'], d['ms_per_step'], 'frac', r['frac'], {k:v['TFLOP/s'] for k,v in r['by_pass'].items()}, 'gn', r.get('hbm_kernels',{}).get('ms_per_step'))"
done
