#!/bin/bash
# last call of the round: GPU test suite + smoke on the final build, then the C4 re-tune confirmation
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rc=0; timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/t4_tests.log 2>&1 || rc=$?
tail -2 gpurun_out/t4_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t4_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/t4_smoke.log
bash tools/r4_c4ab.sh
