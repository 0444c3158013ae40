#!/bin/bash
# attention-backward LDS overlay (dS over V's staging) on / off (xlib/lib_noovl.so), C5 and C2, same box
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { tag=$1; shift; cfg=$1; shift; env "$@" timeout -k 10 300 python bench.py $cfg --no-cpu-baseline --no-gpu-only > gpurun_out/ovl_$tag.json 2> gpurun_out/ovl_$tag.err || { tail -20 gpurun_out/ovl_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/ovl_$tag.json').read().strip().splitlines()[-1]);print('$tag',d['value'],d['ms_per_step'])"; }
for i in 1 2 3; do
run c5_ovl_$i "--config c5" ERGM_NONE=1
run c5_noovl_$i "--config c5" ERGM_LIB_PATH=xlib/lib_noovl.so
done
for i in 1 2; do
run c2_ovl_$i "" ERGM_NONE=1
run c2_noovl_$i "" ERGM_LIB_PATH=xlib/lib_noovl.so
done
