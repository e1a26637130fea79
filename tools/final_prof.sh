#!/bin/bash
# Round-end evidence for HEAD, in two calls (each within gpurun's limit):
#   tools/final_prof.sh <tag> a : PMC FETCH_SIZE / WRITE_SIZE passes of the GEMM family on c4 (-> the traffic file the
#                                 bench lines then report), bench lines c4 (--detail), c2, c3
#   tools/final_prof.sh <tag> b : bench lines c5, c1; rocprofv3 kernel stats of c4 / c2 / c3 (3 steps, no warm-up)
TAG=${1:-r02}; PART=${2:-a}; RND=${RND:-r02}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
bench() {
  timeout -k 10 400 python -u bench.py --config $1 --steps 10 --warmup 3 --detail > gpurun_out/$TAG/bench_$1.json 2> gpurun_out/$TAG/bench_$1.err || exit $?
  cut -c1-200 gpurun_out/$TAG/bench_$1.json
}
if [ "$PART" = a ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --pmc $C --kernel-include-regex gemm3x -d gpurun_out/traffic_c4_$C -o run --output-format csv -- python3 bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timing > gpurun_out/$TAG/traffic_c4_$C.log 2>&1 || exit $?
  done
  python3 tools/pmc_traffic.py c4 $RND && cp profiles/${RND}_c4_gemm_traffic.json gpurun_out/$TAG/ || exit 1
  for c in c4 c2 c3; do bench $c; done
else
  for c in c5 c1; do bench $c; done
  for c in c4 c2 c3; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 0 --no-cpu-baseline --no-kernel-timing > gpurun_out/$TAG/prof_$c.log 2>&1 || exit $?
  done
fi
