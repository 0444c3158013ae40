#!/bin/bash
# Forward knock-outs (experiment library xlib/lib_ko.so, ERGM_X_KO = mask of fwd_block launch groups skipped;
# results wrong, timing only): how much of the forward's time each launch group holds.
# groups: 0 LN1, 1 c_attn, 2 attention, 3 attn c_proj, 4 LN_x, 5 q, 6 cross-attention, 7 cross c_proj, 8 LN2,
# 9 c_fc, 10 mlp c_proj
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export ERGM_LIB_PATH=xlib/lib_ko.so
run() { tag=$1; m=$2; ERGM_X_KO=$m ERGM_BENCH_PHASES=gpurun_out/ko_ph_$tag.json timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/ko_$tag.json 2> gpurun_out/ko_$tag.err || { tail -20 gpurun_out/ko_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/ko_$tag.json').read().strip().splitlines()[-1]);p=json.load(open('gpurun_out/ko_ph_$tag.json'));print('$tag',d['ms_per_step'],round(p['forward_ms'],3),round(p['backward_opt_ms'],3))"; }
for i in 1 2; do
run none_$i 0
run q_$i 32
run selfattn_$i 4
run crossattn_$i 64
run lnx_ln2_$i 272
run cattn_$i 2
run resid3_$i 1160
done
