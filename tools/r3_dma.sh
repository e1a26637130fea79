#!/bin/bash
# bf16 LDS-DMA path check: its numerics tests, then the c5 bench line (+ optional extra configs)
TAG=${1:-dma}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest ${DMA_TESTS:-tests/test_gpu_bf16_dma.py tests/test_gpu_c5.py tests/test_gpu_bench_geometry.py tests/test_gpu_parity.py} -m gpu -v -x --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/$TAG/pytest.log | tail -30
[ $rc -eq 0 ] || exit $rc
for c in "$@"; do
  timeout -k 10 300 python -u bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/$TAG/bench_$c.json 2> gpurun_out/$TAG/bench_$c.err || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/$TAG/bench_$c.json')); r=d['roofline']
print('$c', d['value'], d['ms_per_step'], 'frac', r['frac'], {k:(v['TFLOP/s'],v['ms']) for k,v in r['by_pass'].items()}, 'gn', r.get('hbm_kernels',{}).get('ms_per_step'))"
done
