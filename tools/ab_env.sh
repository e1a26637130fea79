#!/bin/bash
# In-call A/B of environment switches on the c4 bench (same box, interleaved): tools/ab_env.sh <tag> "<envA>" "<envB>" ...
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
  i=0
  for e in "$@"; do
    env $e timeout -k 10 300 python -u bench.py --config ${CFG:-c4} --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_${i}_$r.json 2> gpurun_out/${TAG}_${i}_$r.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], {k: v['TFLOP/s'] for k, v in r['by_pass'].items()})" gpurun_out/${TAG}_${i}_$r.json "$e"
    i=$((i+1))
  done
done
