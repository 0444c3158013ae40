#!/bin/bash
# short attention backward with its per-query arrays below 64 KiB of LDS and the LSE pre-scaled: parity, isolated
# timing, and an interleaved C2 A/B against the previous library (xlib/lib_prev.so)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_dropout.py -x -q --timeout 240 --timeout-method thread -k "attn or attention or fused or small or c2 or dropout or deterministic or maximum or odd" > gpurun_out/al_tests.log 2>&1 || { tail -40 gpurun_out/al_tests.log; exit 1; }
tail -2 gpurun_out/al_tests.log
timeout -k 10 120 python tools/attn_bench.py --only c2 2>&1 | grep -v amdgpu.ids
ERGM_LIB_PATH=xlib/lib_prev.so timeout -k 10 120 python tools/attn_bench.py --only c2 2>&1 | grep -v amdgpu.ids
run() { tag=$1; shift; env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/al_$tag.json 2> gpurun_out/al_$tag.err || { tail -20 gpurun_out/al_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/al_$tag.json').read().strip().splitlines()[-1]);print('$tag',d['value'],d['ms_per_step'])"; }
for i in 1 2 3; do
run prev_$i ERGM_LIB_PATH=xlib/lib_prev.so
run new_$i ERGM_NONE=1
done
