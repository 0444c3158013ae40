#!/bin/bash
# backward knock-outs (experiment library xlib/lib_bko.so, ERGM_X_BKO mask; results wrong, timing only):
# 1 LM-head dW (side stream), 2 LayerNorm parameter reduces (side), 4 every AdamW range (optimizer stream),
# 8 the attention backward (data-gradient chain)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export ERGM_LIB_PATH=xlib/lib_bko.so
run() { tag=$1; m=$2; ERGM_X_BKO=$m ERGM_BENCH_PHASES=gpurun_out/bko_ph_$tag.json timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/bko_$tag.json 2> gpurun_out/bko_$tag.err || { tail -20 gpurun_out/bko_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/bko_$tag.json').read().strip().splitlines()[-1]);p=json.load(open('gpurun_out/bko_ph_$tag.json'));print('$tag',d['ms_per_step'],round(p['forward_ms'],3),round(p['backward_opt_ms'],3))"; }
for i in 1 2; do
run none_$i 0
run lmdw_$i 1
run lnred_$i 2
run adamw_$i 4
run attn_$i 8
done
