#!/bin/bash
# Fused AdamW (weight-gradient epilogue + LayerNorm reduce): the new bitwise tests, the model / op suites, then
# alternating C2 bench runs fused vs per-range passes.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 240 --timeout-method thread -k "adamw or fused or overlapped or grouped or chains or c2 or small" > gpurun_out/r4f_tests.log 2>&1 || { tail -40 gpurun_out/r4f_tests.log; exit 1; }
tail -3 gpurun_out/r4f_tests.log
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/r4f_$tag.json 2> gpurun_out/r4f_$tag.err || { tail -20 gpurun_out/r4f_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/r4f_$tag.json').read().strip().splitlines()[-1]);print('$tag',d['value'],d['ms_per_step'],d['roofline']['achieved'],d.get('gpu_only_ms_per_step'))"; }
run fused1
run plain1 --no-fuse-optim
run fused2
run plain2 --no-fuse-optim
run keep1 --keep-grads
