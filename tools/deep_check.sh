#!/bin/bash
# Deep (two-tile) prefetch for small GEMM tiles + the fastcall host path: full GPU suite, then c3 / c2 / c1 benches
# with and without the fastcall module (MVAE_NO_FASTCALL=1), interleaved.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/deep_tests.log 2>&1 || { tail -30 gpurun_out/deep_tests.log; exit 1; }
tail -2 gpurun_out/deep_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/deep_smoke.log 2>&1 || { tail -5 gpurun_out/deep_smoke.log; exit 1; }
tail -1 gpurun_out/deep_smoke.log
one() {  # <tag> <config> [env]
  env $3 timeout -k 10 300 python -u bench.py --config $2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/dp_$1.json 2> gpurun_out/dp_$1.err || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['gemm_ms_per_step'], {k: v['TFLOP/s'] for k, v in r['by_pass'].items()})" gpurun_out/dp_$1.json "$1"
}
for r in 1 2; do
  one c3_fast_$r c3
  one c3_ctypes_$r c3 MVAE_NO_FASTCALL=1
done
one c2 c2
one c1 c1
one c4 c4
