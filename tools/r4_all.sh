#!/bin/bash
# round-4 closing run: the GPU test suite, then the judged measurements (tools/r4_final.sh)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rc=0; timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/t4_tests.log 2>&1 || rc=$?
tail -3 gpurun_out/t4_tests.log
# test failures (1) still let the measurements run; a crash, abort or time limit ends the script
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t4_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/t4_smoke.log
bash tools/r4_final.sh
