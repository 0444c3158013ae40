#!/bin/bash
# Kernel trace + stats of the C2 bench (rocprofv3), the per-step breakdown, and the DP rehearsal
# (two self-launched ranks on the one GPU over gloo).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=${1:-cur}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-only > gpurun_out/prof_$TAG.log 2>&1
python tools/trace_step.py gpurun_out/prof_$TAG 40 --phases > gpurun_out/step_$TAG.txt 2>&1 || true
python tools/prof_summary.py gpurun_out/prof_$TAG 0 40 > gpurun_out/stats_$TAG.txt 2>&1 || true
rm -f gpurun_out/prof_$TAG/run_kernel_trace.csv.gz
if [ "${2:-}" = "rehearse" ]; then
  ERGM_BENCH_REHEARSE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/rehearse.log 2>&1
  tail -2 gpurun_out/rehearse.log
fi
tail -1 gpurun_out/prof_$TAG.log | cut -c1-300
