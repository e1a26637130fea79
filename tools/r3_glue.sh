#!/bin/bash
# GPU check of the fused step glue: its tests + the golden / graph / loss tests, c3 and c4 bench lines and the c3
# per-step kernel table.   tools/r3_glue.sh <tag> [extra test files]
TAG=${1:-g}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests/test_gpu_fused_glue.py tests/test_gpu_parity.py tests/test_gpu_graph.py \
  tests/test_gpu_losses.py tests/test_gpu_latent.py "$@" -m gpu -q -x --timeout 300 --timeout-method thread \
  > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/$TAG/pytest.log
[ $rc -eq 0 ] || exit $rc
for c in c3 c4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG/bench_$c.json 2> gpurun_out/$TAG/bench_$c.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_$c.json')); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], {k:v['TFLOP/s'] for k,v in r['by_pass'].items()})"
done
bash tools/prof_diff.sh $TAG c3 2 12
