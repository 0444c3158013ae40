#!/bin/bash
# forward residual GEMMs with split-K (separate reduce launch applying the epilogue), in-step: does a shorter K loop
# per workgroup shorten the latency-bound forward?  (runtime overrides; forward device time via ERGM_BENCH_PHASES)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { tag=$1; shift; ERGM_BENCH_PHASES=gpurun_out/sr_ph_$tag.json timeout -k 10 200 python tools/bench_override.py "$@" -- --no-cpu-baseline --no-gpu-only > gpurun_out/sr_$tag.json 2> gpurun_out/sr_$tag.err || { tail -20 gpurun_out/sr_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/sr_$tag.json').read().strip().splitlines()[-1]);p=json.load(open('gpurun_out/sr_ph_$tag.json'));print('$tag',d['ms_per_step'],round(p['forward_ms'],3))"; }
for i in 1 2; do
run base_$i
run mlp_s2_$i 1024,768,3072,0,1,0,2
run mlp_s3_$i 1024,768,3072,0,1,0,3
run all_s2_$i 1024,768,3072,0,1,0,2 1024,768,768,0,1,0,2
done
