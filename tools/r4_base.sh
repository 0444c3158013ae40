#!/bin/bash
# Round-4 baseline on a fresh box: GPU suite + C2 bench (HEAD of the round start).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4b_tests.log 2>&1 || rc=$?
tail -3 gpurun_out/r4b_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4b_bench.json 2> gpurun_out/r4b_bench.err
tail -c 300 gpurun_out/r4b_bench.json
