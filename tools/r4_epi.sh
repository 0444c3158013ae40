#!/bin/bash
# AdamW epilogue as its own instantiations: the AdamW / fused-optimizer parity tests, then C5 and C2 against the
# round-3 tree (xold) on the same box
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 240 --timeout-method thread -k "adamw or fused_optimizer or gemm or grouped or overlapped" > gpurun_out/epi_tests.log 2>&1 || { tail -40 gpurun_out/epi_tests.log; exit 1; }
tail -2 gpurun_out/epi_tests.log
run() { tag=$1; dir=$2; shift; shift; (cd $dir && timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-gpu-only > $GRAFT_REPO_ROOT/gpurun_out/epi_$tag.json 2> $GRAFT_REPO_ROOT/gpurun_out/epi_$tag.err) || { tail -20 gpurun_out/epi_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/epi_$tag.json').read().strip().splitlines()[-1]);print('$tag',d['value'],d['ms_per_step'])"; }
for i in 1 2; do
run c5_r3_$i xold --config c5
run c5_r4_$i . --config c5
run c2_r3_$i xold
run c2_r4_$i .
done
run c2_fuse_r4 . --fuse-optim
