#!/bin/bash
# forward chain offset (experiment library xlib/lib_off.so): the second chain starts after the first chain's first
# ERGM_X_OFF launch groups, so the two chains' heavy GEMMs stop coinciding
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export ERGM_LIB_PATH=xlib/lib_off.so
run() { tag=$1; m=$2; ERGM_X_OFF=$m ERGM_BENCH_PHASES=gpurun_out/off_ph_$tag.json timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/off_$tag.json 2> gpurun_out/off_$tag.err || { tail -20 gpurun_out/off_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/off_$tag.json').read().strip().splitlines()[-1]);p=json.load(open('gpurun_out/off_ph_$tag.json'));print('$tag',d['ms_per_step'],round(p['forward_ms'],3),round(p['backward_opt_ms'],3))"; }
for i in 1 2; do
run o0_$i 0
run o3_$i 3
run o6_$i 6
run o11_$i 11
done
