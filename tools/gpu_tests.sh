#!/bin/bash
# the whole GPU test suite (round-4 state)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rc=0; timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/t4_tests.log 2>&1 || rc=$?
tail -15 gpurun_out/t4_tests.log
exit $rc
