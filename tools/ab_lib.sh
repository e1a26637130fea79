#!/bin/bash
# In-call A/B of library variants (variants/<name>/libmvae_hip.so) on a bench config: tools/ab_lib.sh <tag> <v1> <v2> ...
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
  for v in "$@"; do
    MVAE_HIP_LIB=variants/$v/libmvae_hip.so timeout -k 10 300 python -u bench.py --config ${CFG:-c4} --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_${v}_$r.json 2> gpurun_out/${TAG}_${v}_$r.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; h=r['hbm_kernels']; print(sys.argv[2], d['value'], {k: v['TFLOP/s'] for k, v in r['by_pass'].items()}, h['ms_per_step'], {k: (v['ms'], v['GB/s']) for k, v in h['by_pass'].items()})" gpurun_out/${TAG}_${v}_$r.json "$v"
  done
done
