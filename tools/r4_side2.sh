#!/bin/bash
# a second weight-gradient stream (experiment library xlib/lib_s2.so, ERGM_X_SIDE2=1: every other dW flush runs
# there and the side stream joins it at each stage mark), C2, interleaved
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export ERGM_LIB_PATH=xlib/lib_s2.so
run() { tag=$1; m=$2; ERGM_X_SIDE2=$m ERGM_BENCH_PHASES=gpurun_out/s2_ph_$tag.json timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/s2_$tag.json 2> gpurun_out/s2_$tag.err || { tail -20 gpurun_out/s2_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/s2_$tag.json').read().strip().splitlines()[-1]);p=json.load(open('gpurun_out/s2_ph_$tag.json'));print('$tag',d['ms_per_step'],round(p['forward_ms'],3),round(p['backward_opt_ms'],3))"; }
for i in 1 2 3; do
run one_$i 0
run two_$i 1
done
