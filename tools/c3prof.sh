cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c3a.json 2> gpurun_out/c3a.err || exit $?
cut -c1-600 gpurun_out/c3a.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c3prof -o run --output-format csv -- python bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > gpurun_out/c3prof.log 2>&1 || exit $?
