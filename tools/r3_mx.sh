#!/bin/bash
# MX-fp8 (config 5): quantiser / GEMM tests, the fp8 model gates on the MX path, then C5 benches: MX vs the per-row
# / per-column fp8 path vs bf16.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_mx.py tests/test_gpu_fp8.py -x -q --timeout 180 --timeout-method thread > gpurun_out/t_mx.log 2>&1 || { tail -40 gpurun_out/t_mx.log; exit 1; }
tail -2 gpurun_out/t_mx.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_c5.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_mx_c5.log 2>&1 || { tail -40 gpurun_out/t_mx_c5.log; exit 1; }
tail -2 gpurun_out/t_mx_c5.log
run() { tag=$1; args=$2; shift 2; env "$@" timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline --no-gpu-only $args > gpurun_out/mx_$tag.json 2>gpurun_out/mx_$tag.err || { echo "$tag FAILED"; tail -3 gpurun_out/mx_$tag.err; return; }; echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/mx_$tag.json'));print(d['value'],d['ms_per_step'],d['train_metrics'])")"; }
for r in 1 2; do run mx$r "" ERGM_FP8_MX=1; run row$r "" ERGM_FP8_MX=0; run bf16_$r --no-fp8 ERGM_NONE=1; done
