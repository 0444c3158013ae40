#!/bin/bash
# C2 sanity after the C4 table entries: previous vs current library, interleaved
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/c2c_$tag.json 2> gpurun_out/c2c_$tag.err || { tail -20 gpurun_out/c2c_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/c2c_$tag.json').read().strip().splitlines()[-1]);print('$tag',d['value'],d['ms_per_step'],d['host_enqueue_ms_per_step_in_timed_loop'])"; }
for i in 1 2; do
run prev_$i ERGM_LIB_PATH=xlib/lib_prev.so
run new_$i ERGM_NONE=1
done
