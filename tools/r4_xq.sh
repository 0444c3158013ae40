#!/bin/bash
# query projection inside the cross-attention forward: parity (bitwise vs two launches + the oracle tests), then an
# interleaved C2 A/B (ERGM_XQ_FUSE=0 / 1) with the forward's device time
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_dropout.py tests/test_gpu_generate.py -x -q --timeout 240 --timeout-method thread -k "fused_cross or small or c2 or dropout or deterministic or odd or maximum or generate or decode" > gpurun_out/xq_tests.log 2>&1 || { tail -40 gpurun_out/xq_tests.log; exit 1; }
tail -2 gpurun_out/xq_tests.log
run() { tag=$1; shift; env "$@" ERGM_BENCH_PHASES=gpurun_out/xq_ph_$tag.json timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/xq_$tag.json 2> gpurun_out/xq_$tag.err || { tail -20 gpurun_out/xq_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/xq_$tag.json').read().strip().splitlines()[-1]);p=json.load(open('gpurun_out/xq_ph_$tag.json'));print('$tag',d['value'],d['ms_per_step'],round(p['forward_ms'],3))"; }
for i in 1 2 3; do
run off_$i ERGM_XQ_FUSE=0
run on_$i ERGM_XQ_FUSE=1
done
