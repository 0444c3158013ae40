#!/bin/bash
# Knob sweep on the C2 step: AdamW grid caps, data-gradient GEMM configurations of the critical chain.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
b() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only "$@" > gpurun_out/x3_$tag.json 2> gpurun_out/x3_$tag.err || { tail -5 gpurun_out/x3_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/x3_$tag.json').read().strip().splitlines()[-1]);print('$tag',d['value'],d['ms_per_step'])"; }
o() { tag=$1; ov=$2; timeout -k 10 200 python tools/bench_override.py $ov -- --no-cpu-baseline --no-gpu-only > gpurun_out/x3_$tag.json 2> gpurun_out/x3_$tag.err || { tail -5 gpurun_out/x3_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/x3_$tag.json').read().strip().splitlines()[-1]);print('$tag',d['value'],d['ms_per_step'])"; }
# fc dX: 2048,768,3072 MK NK ; c_attn dX: 2048,768,2304 ; GELU' dX: 2048,3072,768 ; d_o dX 2048,768,768 (bf16)
for r in 1 2; do
b base$r
b cap2048_$r --adamw-blocks 2048
b cap1024_$r --adamw-blocks 1024
o dx0_$r "2048,768,3072,0,0,0,1 2048,768,2304,0,0,0,1"
o dx33_$r "2048,768,3072,0,0,33,1 2048,768,2304,0,0,33,1"
o dx14_$r "2048,768,3072,0,0,14,1 2048,768,2304,0,0,14,1"
o gelu2_$r "2048,3072,768,0,0,2,1"
done
