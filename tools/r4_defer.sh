#!/bin/bash
# AdamW of blocks 1..L-1 deferred into the next forward (bench --defer-update) vs per-bucket during the backward
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { tag=$1; shift; ERGM_BENCH_PHASES=gpurun_out/df_ph_$tag.json timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only "$@" > gpurun_out/df_$tag.json 2> gpurun_out/df_$tag.err || { tail -20 gpurun_out/df_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/df_$tag.json').read().strip().splitlines()[-1]);p=json.load(open('gpurun_out/df_ph_$tag.json'));print('$tag',d['value'],d['ms_per_step'],round(p['forward_ms'],3),round(p['backward_opt_ms'],3))"; }
for i in 1 2 3; do
run base_$i
run defer_$i --defer-update
done
