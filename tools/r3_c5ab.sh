#!/bin/bash
# C5 confirmation runs (alternating): MX-fp8 default, bf16, MX + fp8 backward; then smoke().
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { tag=$1; args=$2; shift 2; env "$@" timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline --no-gpu-only $args > gpurun_out/ab5_$tag.json 2>gpurun_out/ab5_$tag.err || { echo "$tag FAILED"; tail -3 gpurun_out/ab5_$tag.err; exit 1; }; echo "$tag $(python -c "import json;d=json.loads(open('gpurun_out/ab5_$tag.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"; }
for r in 1 2; do run mx$r "" ERGM_NONE=1; run bf16_$r --no-fp8 ERGM_NONE=1; run mxb$r "" ERGM_FP8_BWD=1; done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
