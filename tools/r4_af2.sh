#!/bin/bash
# attention backward LDS overlay (83 KiB) and the fused dO GEMM: parity, then interleaved C2 A/B against the previous
# commit's library (xlib/lib_old.so)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_dropout.py tests/test_gpu_ops.py -x -q --timeout 240 --timeout-method thread -k "fused_attention or small or c2 or chains or dropout or deterministic or attn or odd or maximum" > gpurun_out/af2_tests.log 2>&1 || { tail -40 gpurun_out/af2_tests.log; exit 1; }
tail -2 gpurun_out/af2_tests.log
run() { tag=$1; shift; env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/af2_$tag.json 2> gpurun_out/af2_$tag.err || { tail -20 gpurun_out/af2_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/af2_$tag.json').read().strip().splitlines()[-1]);print('$tag',d['value'],d['ms_per_step'])"; }
for i in 1 2 3; do
run old_$i ERGM_LIB_PATH=xlib/lib_old.so
run ovl_$i ERGM_ATTN_FUSE=0
run fused_$i ERGM_ATTN_FUSE=1
done
