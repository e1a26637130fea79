#!/bin/bash
# c4 bench A/B of GroupNorm library variants (variants/<name>/libmvae_hip.so; "default" = in-tree), interleaved:
# prints the GN fwd / bwd chain bandwidth of each run.   usage: tools/ab_gn_c4.sh <tag> <variant> ...
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = default ]; then unset MVAE_HIP_LIB; else export MVAE_HIP_LIB=variants/$v/libmvae_hip.so; fi
    timeout -k 10 300 python -u bench.py --config ${CFG:-c4} --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_${v}_$r.json 2> gpurun_out/${TAG}_${v}_$r.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); h=d['roofline']['hbm_kernels']; print(sys.argv[2], d['value'], h['frac'], {k: (v['ms'], v['GB/s']) for k, v in h['by_pass'].items()})" gpurun_out/${TAG}_${v}_$r.json "$v"
  done
done
