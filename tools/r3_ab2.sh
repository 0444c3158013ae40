#!/bin/bash
# emotion-head / LayerNorm-backward LDS changes vs HEAD's library (ab/lib_old.so), and the 8-wave IL GEMM
# overrides in-step.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 180 --timeout-method thread -k "layernorm or emotion or full_c2 or tiny or small" > gpurun_out/t_ab2.log 2>&1 || { tail -40 gpurun_out/t_ab2.log; exit 1; }
tail -2 gpurun_out/t_ab2.log
run() { tag=$1; shift; env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/ab_$tag.json 2>/dev/null || exit 1; echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/ab_$tag.json'));print(d['value'],d['ms_per_step'])")"; }
for i in 1 2 3; do run old$i ERGM_LIB_PATH=ab/lib_old.so; run new$i ERGM_NONE=1; done
ROUNDS=2 bash tools/ab_override.sh "base:" \
 "il30:1024,3072,768,0,1,30,1 2048,3072,768,0,0,30,1 2048,18432,768,0,1,30,1 1024,2304,768,0,1,27,1" 2>&1 | grep -v amdgpu.ids
