#!/bin/bash
# Split-K conv planner: kernel + parity tests, then c2 / c1 / c4 bench A/B against MVAE_NO_CONV_SPLITK=1.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sk_tests.log 2>&1 || { tail -30 gpurun_out/sk_tests.log; exit 1; }
tail -2 gpurun_out/sk_tests.log
one() {  # <tag> <config> [env]
  env $3 timeout -k 10 300 python -u bench.py --config $2 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/sk_$1.json 2> gpurun_out/sk_$1.err || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], {k: v['TFLOP/s'] for k, v in r['by_pass'].items()})" gpurun_out/sk_$1.json "$1"
}
for r in 1 2; do
  one c2_on_$r c2
  one c2_off_$r c2 MVAE_NO_CONV_SPLITK=1
done
one c1_on c1
one c1_off c1 MVAE_NO_CONV_SPLITK=1
one c4_on c4
one c4_off c4 MVAE_NO_CONV_SPLITK=1
