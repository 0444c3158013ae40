#!/bin/bash
# C4 / C5 with and without the round-4 fusions (same box, interleaved)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { tag=$1; shift; cfgarg=$1; shift; env "$@" timeout -k 10 300 python bench.py $cfgarg --no-cpu-baseline --no-gpu-only > gpurun_out/c45_$tag.json 2> gpurun_out/c45_$tag.err || { tail -20 gpurun_out/c45_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/c45_$tag.json').read().strip().splitlines()[-1]);print('$tag',d['value'],d['ms_per_step'])"; }
for i in 1 2; do
run c5_$i "--config c5" ERGM_NONE=1
run c5_noaf_$i "--config c5" ERGM_ATTN_FUSE=0
run c5bf_$i "--config c5 --no-fp8" ERGM_NONE=1
run c5bf_nofuse_$i "--config c5 --no-fp8" ERGM_ATTN_FUSE=0 ERGM_XQ_FUSE=0
run c4_$i "--config c4" ERGM_NONE=1
run c4_noxq_$i "--config c4" ERGM_XQ_FUSE=0
done
