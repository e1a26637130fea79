#!/bin/bash
# Deep-prefetch A/B (variants/deep vs variants/nodeep) on the per-shape GEMM time of c3 / c2 / c1 (instrumented step)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for c in c3 c1 c2; do
  for r in 1 2; do
    for v in deep nodeep; do
      MVAE_HIP_LIB=variants/$v/libmvae_hip.so timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --detail > gpurun_out/ab_${c}_${v}_$r.json 2> gpurun_out/ab_${c}_${v}_$r.err || exit $?
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], r['gemm_ms_per_step'], {k: v['ms'] for k, v in r['by_pass'].items()})" gpurun_out/ab_${c}_${v}_$r.json "$c $v $r"
    done
  done
done
