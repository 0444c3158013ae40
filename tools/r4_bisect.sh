#!/bin/bash
# C5 regression bisection: round-3 tree (xold), first round-4 commit 4d3ca2c (xold2), current without / with the
# fused attention backward
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { tag=$1; dir=$2; shift; shift; (cd $dir && env "$@" timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-gpu-only > $GRAFT_REPO_ROOT/gpurun_out/bis_$tag.json 2> $GRAFT_REPO_ROOT/gpurun_out/bis_$tag.err) || { tail -20 gpurun_out/bis_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/bis_$tag.json').read().strip().splitlines()[-1]);print('$tag',d['value'],d['ms_per_step'])"; }
for i in 1 2; do
run r3_$i xold ERGM_NONE=1
run c1_$i xold2 ERGM_NONE=1
run cur_noaf_$i . ERGM_ATTN_FUSE=0
run cur_$i . ERGM_NONE=1
done
