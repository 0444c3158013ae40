#!/bin/bash
# fp8 data-gradient GEMMs (config 5, ERGM_FP8_BWD): MX tests, the C5 model gates, then C5 benches:
# MX fwd+bwd (default) vs MX forward only vs bf16.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_mx.py -x -q --timeout 180 --timeout-method thread > gpurun_out/t_mxb.log 2>&1 || { tail -40 gpurun_out/t_mxb.log; exit 1; }
tail -1 gpurun_out/t_mxb.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_c5.py -x -q -rA --timeout 300 --timeout-method thread > gpurun_out/t_mxb_c5.log 2>&1 || { tail -60 gpurun_out/t_mxb_c5.log; exit 1; }
tail -1 gpurun_out/t_mxb_c5.log
run() { tag=$1; args=$2; shift 2; env "$@" timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline --no-gpu-only $args > gpurun_out/mxb_$tag.json 2>gpurun_out/mxb_$tag.err || { echo "$tag FAILED"; tail -3 gpurun_out/mxb_$tag.err; return; }; echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/mxb_$tag.json'));print(d['value'],d['ms_per_step'],d['train_metrics'])")"; }
timeout -k 10 200 python tools/mx_shapes.py 2048 > gpurun_out/mxs2.log 2>&1
for r in 1 2; do run mxf$r "" ERGM_FP8_BWD=0; run mxb$r "" ERGM_FP8_BWD=1; run row$r "" ERGM_FP8_MX=0; run bf16_$r --no-fp8 ERGM_NONE=1; done
