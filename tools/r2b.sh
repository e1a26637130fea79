#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./tools/micro/hbm_stream > gpurun_out/micro_hbm.txt 2>&1 || exit $?
cat gpurun_out/micro_hbm.txt
timeout -k 10 300 python -u tools/torch_prof.py --config c3 > gpurun_out/tprof_c3.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/torch_prof.py --config c1 > gpurun_out/tprof_c1.txt 2>&1 || exit $?
