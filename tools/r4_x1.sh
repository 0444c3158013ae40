#!/bin/bash
# Experiment: where does the fused optimizer's slowdown come from?  Interleaved C2 runs of
#   plain (per-range AdamW), plain + late fork, fused without the epilogue update (knock-out, results wrong),
#   fused (current).  xlib/lib_x.so = the library with ERGM_X_LATE / ERGM_X_EPI experiment knobs.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export ERGM_LIB_PATH=xlib/lib_x.so
run() { tag=$1; shift; env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only $BA > gpurun_out/x1_$tag.json 2> gpurun_out/x1_$tag.err || { tail -20 gpurun_out/x1_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/x1_$tag.json').read().strip().splitlines()[-1]);print('$tag',d['value'],d['ms_per_step'],d['roofline']['achieved'])"; }
for i in 1 2; do
BA= run plain$i ERGM_NONE=1
BA= run plainlate$i ERGM_X_LATE=1
BA=--fuse-optim run fuse_noepi$i ERGM_X_EPI=0
BA=--fuse-optim run fuse_early$i ERGM_X_LATE=0
BA=--fuse-optim run fuse$i ERGM_NONE=1
done
# GPU-only kernel trace of the plain step (the bench's last steps run behind a spin kernel: no host in the loop)
unset ERGM_LIB_PATH
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/x1_prof -o run --output-format csv -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/x1_prof.log 2>&1
python tools/timeline.py gpurun_out/x1_prof --step -2 --min-us 5 > gpurun_out/x1_timeline.txt 2>&1 || true
python tools/trace_step.py gpurun_out/x1_prof 40 > gpurun_out/x1_trace_step.txt 2>&1 || true
rm -f gpurun_out/x1_prof/run_kernel_trace.csv.gz
head -5 gpurun_out/x1_timeline.txt
