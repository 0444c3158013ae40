#!/bin/bash
# The GPU test suite (optionally a -k expression as $1), then one C2 bench line.  Logs under gpurun_out/.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
K=${1:+-k "$1"}
rc=0; eval timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $K > gpurun_out/tests.log 2>&1 || rc=$?
grep -E "passed|failed|error" gpurun_out/tests.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
tail -c 600 gpurun_out/bench_c2.json
