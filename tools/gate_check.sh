#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gate_tests.log 2>&1 || { tail -30 gpurun_out/gate_tests.log; exit 1; }
tail -2 gpurun_out/gate_tests.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/gate_c3_$r.json 2>/dev/null || exit $?
  cut -c1-160 gpurun_out/gate_c3_$r.json
done
timeout -k 10 300 python -u tools/torch_prof.py --config c3 > gpurun_out/tprof_c3b.txt 2>&1 || exit $?
grep -E "Self CPU time total|Self CUDA time total|FiniteGate" gpurun_out/tprof_c3b.txt
