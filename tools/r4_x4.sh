#!/bin/bash
# Weight-gradient fork timing and optimizer lag (xlib/lib_x.so: ERGM_X_EAGER = each dW GEMM forked and launched as
# soon as its dY is formed, no pairing; ERGM_X_LAG = stages between a block's backward and its AdamW).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export ERGM_LIB_PATH=xlib/lib_x.so
run() { tag=$1; shift; env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/x4_$tag.json 2> gpurun_out/x4_$tag.err || { tail -20 gpurun_out/x4_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/x4_$tag.json').read().strip().splitlines()[-1]);print('$tag',d['value'],d['ms_per_step'])"; }
for i in 1 2; do
run base$i ERGM_NONE=1
run eager$i ERGM_X_EAGER=1
run lag1_$i ERGM_X_LAG=1
run lag3_$i ERGM_X_LAG=3
run lag4_$i ERGM_X_LAG=4
run eager_lag3_$i ERGM_X_EAGER=1 ERGM_X_LAG=3
done
