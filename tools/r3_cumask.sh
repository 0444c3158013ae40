#!/bin/bash
# CU-mask experiments: the weight-gradient / optimizer streams (and optionally the caller's stream) restricted to
# subsets of the CUs (hipExtStreamCreateWithCUMask); C2 bench, two sequential rounds.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
source tools/cumasks.env
run() { tag=$1; shift; env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/cm_$tag.json 2> gpurun_out/cm_$tag.err || { echo "$tag FAILED"; tail -3 gpurun_out/cm_$tag.err; return; }; echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/cm_$tag.json'));print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])")"; }
for r in 1 2; do
run base$r ERGM_NONE=1
run sodd$r ERGM_SIDE_CUMASK=$ODD ERGM_OPT_CUMASK=$ODD
run shi$r ERGM_SIDE_CUMASK=$HI ERGM_OPT_CUMASK=$HI
run sq1$r ERGM_SIDE_CUMASK=$Q1 ERGM_OPT_CUMASK=$Q1
run sq3$r ERGM_SIDE_CUMASK=$Q3 ERGM_OPT_CUMASK=$Q3
run part$r ERGM_SIDE_CUMASK=$ODD ERGM_OPT_CUMASK=$ODD ERGM_MAIN_CUMASK=$EVEN
run partq$r ERGM_SIDE_CUMASK=$Q1 ERGM_OPT_CUMASK=$Q1 ERGM_MAIN_CUMASK=$Q3
done
