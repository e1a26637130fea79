#!/bin/bash
# GPU check of the fused disentangled glue: its tests + the golden / graph / loss tests, a c3 bench line and the c3
# per-step kernel table.   tools/r3_glue.sh <tag>
TAG=${1:-g}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest tests/test_gpu_fused_glue.py tests/test_gpu_parity.py tests/test_gpu_graph.py \
  tests/test_gpu_losses.py tests/test_gpu_latent.py -m gpu -q -x --timeout 300 --timeout-method thread \
  > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/$TAG/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG/bench_c3.json 2> gpurun_out/$TAG/bench_c3.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench_c3.json')); print('c3', d['value'], d['ms_per_step'])"
bash tools/prof_diff.sh $TAG c3 2 12
