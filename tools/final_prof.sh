#!/bin/bash
# Round-end evidence for HEAD: bench lines (c4 with --detail, c2, c3, c5, c1), rocprofv3 kernel stats of c4 / c2 / c3,
# PMC FETCH_SIZE / WRITE_SIZE passes of the GEMM family on c4. Usage: tools/final_prof.sh <tag>
TAG=${1:-r02}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
for c in c4 c2 c3 c5 c1; do
  timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 3 --detail > gpurun_out/$TAG/bench_$c.json 2> gpurun_out/$TAG/bench_$c.err || exit $?
  cut -c1-200 gpurun_out/$TAG/bench_$c.json
done
for c in c4 c2 c3; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 0 --no-cpu-baseline --no-kernel-timing > gpurun_out/$TAG/prof_$c.log 2>&1 || exit $?
done
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-include-regex gemm3x -d gpurun_out/traffic_c4_$C -o run --output-format csv -- python3 bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timing > gpurun_out/$TAG/traffic_c4_$C.log 2>&1 || exit $?
done

