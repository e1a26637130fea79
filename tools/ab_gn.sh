#!/bin/bash
# In-call A/B of GroupNorm launch geometry on the c4 bench: tools/ab_gn.sh <tag> "<envA>" "<envB>" ...
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
  i=0
  for e in "$@"; do
    env $e timeout -k 10 300 python -u bench.py --config ${CFG:-c4} --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_${i}_$r.json 2> gpurun_out/${TAG}_${i}_$r.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); h=d['roofline']['hbm_kernels']; print(sys.argv[2], d['value'], h['ms_per_step'], {k: (v['ms'], v['GB/s']) for k, v in h['by_pass'].items()})" gpurun_out/${TAG}_${i}_$r.json "$e"
    i=$((i+1))
  done
done
