#!/bin/bash
# in-step kernel durations with and without the fused attention backward (rocprofv3 kernel trace + stats)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for f in 0 1; do
ERGM_ATTN_FUSE=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/af3_prof$f -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-only > gpurun_out/af3_prof$f.log 2>&1
python tools/prof_summary.py gpurun_out/af3_prof$f 0 40 > gpurun_out/af3_summary$f.txt
done
grep -h "attn_bwd\|64, 64, 2, 2, 4, false, false, 0, true\|total" gpurun_out/af3_summary0.txt gpurun_out/af3_summary1.txt
for f in 0 1; do
ERGM_ATTN_FUSE=$f ERGM_BENCH_PHASES=gpurun_out/af3_phases$f.json timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/af3_b$f.json 2> gpurun_out/af3_b$f.err
cat gpurun_out/af3_phases$f.json; echo
done
