#!/bin/bash
# forward residual / q GEMMs (M = 1024 per forward chain, N = 768, K = 768 | 3072, MK x KN) on the intra-workgroup
# split-K 64x64 tiles (cfg 33: 64 KiB, cfg 34: 96 KiB) vs the automatic 64x64 (cfg 0), in-step, interleaved
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -k "compile or logits" > gpurun_out/fres_tests.log 2>&1 || { tail -40 gpurun_out/fres_tests.log; exit 1; }
tail -2 gpurun_out/fres_tests.log
run() { tag=$1; shift; timeout -k 10 200 python tools/bench_override.py "$@" -- --no-cpu-baseline --no-gpu-only > gpurun_out/fres_$tag.json 2> gpurun_out/fres_$tag.err || { tail -20 gpurun_out/fres_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/fres_$tag.json').read().strip().splitlines()[-1]);print('$tag',d['value'],d['ms_per_step'])"; }
for i in 1 2; do
run base_$i
run c33s_$i 1024,768,768,0,1,33,1
run c33b_$i 1024,768,768,0,1,33,1 1024,768,3072,0,1,33,1
run c34b_$i 1024,768,768,0,1,34,1 1024,768,3072,0,1,34,1
done
