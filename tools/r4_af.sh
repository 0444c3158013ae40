#!/bin/bash
# fused attention backward (c_proj dX GEMM inside attn_bwd_short): parity tests, then an interleaved C2 A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_dropout.py tests/test_gpu_ops.py -x -q --timeout 240 --timeout-method thread -k "fused_attention or small or c2 or chains or dropout or deterministic or attn or odd or maximum" > gpurun_out/af_tests.log 2>&1 || { tail -40 gpurun_out/af_tests.log; exit 1; }
tail -2 gpurun_out/af_tests.log
run() { tag=$1; shift; env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/af_$tag.json 2> gpurun_out/af_$tag.err || { tail -20 gpurun_out/af_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/af_$tag.json').read().strip().splitlines()[-1]);print('$tag',d['value'],d['ms_per_step'])"; }
for i in 1 2 3; do
run off_$i ERGM_ATTN_FUSE=0
run on_$i ERGM_ATTN_FUSE=1
done
