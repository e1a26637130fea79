#!/bin/bash
# Round-3 end evidence at HEAD: the whole GPU suite + smoke, the default bench line (c4 + c2/c3/c5 + parity) and the
# per-step kernel tables of c3 and c4.   tools/r3_final.sh <tag>
TAG=${1:-fin}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/$TAG/pytest.log | head -20; tail -2 gpurun_out/$TAG/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
cut -c1-400 gpurun_out/$TAG/bench.json
bash tools/prof_diff.sh $TAG c3 2 12 > /dev/null || exit $?
bash tools/prof_diff.sh $TAG c4 1 3 > /dev/null || exit $?
head -3 gpurun_out/$TAG/prof_c3_per_step.txt gpurun_out/$TAG/prof_c4_per_step.txt
