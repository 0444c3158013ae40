#!/bin/bash
# C4 re-tune entries against the previous library (xlib/lib_prev.so), C4 and C2, interleaved
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { tag=$1; shift; cfg=$1; shift; env "$@" timeout -k 10 300 python bench.py $cfg --no-cpu-baseline --no-gpu-only > gpurun_out/c4ab_$tag.json 2> gpurun_out/c4ab_$tag.err || { tail -20 gpurun_out/c4ab_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/c4ab_$tag.json').read().strip().splitlines()[-1]);print('$tag',d['value'],d['ms_per_step'])"; }
for i in 1 2; do
run c4_prev_$i "--config c4" ERGM_LIB_PATH=xlib/lib_prev.so
run c4_new_$i "--config c4" ERGM_NONE=1
done
run c2_prev "" ERGM_LIB_PATH=xlib/lib_prev.so
run c2_new "" ERGM_NONE=1
