#!/bin/bash
# Graph-replayed step: full GPU suite (incl. tests/test_gpu_graph.py), smoke, then c3 / c1 / c2 benches graphed vs
# eager (--eager), interleaved, and c4 (eager path, unchanged).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/graph_tests.log 2>&1 || { tail -40 gpurun_out/graph_tests.log; exit 1; }
tail -2 gpurun_out/graph_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/graph_smoke.log 2>&1 || { tail -5 gpurun_out/graph_smoke.log; exit 1; }
one() {  # <tag> <config> [flags]
  timeout -k 10 300 python -u bench.py --config $2 --steps 20 --warmup 5 --no-cpu-baseline $3 > gpurun_out/gr_$1.json 2> gpurun_out/gr_$1.err || { tail -20 gpurun_out/gr_$1.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['step_launch'], d['loss'])" gpurun_out/gr_$1.json "$1"
}
for r in 1 2; do
  one c3_graph_$r c3
  one c3_eager_$r c3 --eager
done
one c1_graph c1
one c1_eager c1 --eager
one c2_graph c2
one c2_eager c2 --eager
