#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in cvae_fwd cvae_fwdbwd cvae_step dis_fwd dis_fwdbwd dis_step; do
  timeout -k 10 120 python -u tools/graph_bisect.py $v > gpurun_out/gb_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; tail -2 gpurun_out/gb_$v.log
  [ $rc -eq 0 ] || exit $rc
done
