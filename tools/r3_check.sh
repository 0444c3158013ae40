#!/bin/bash
# GPU suite + C2 bench + a kernel trace whose last steps are the bench's GPU-only steps (enqueued behind a spin
# kernel, so the trace shows the device timeline without the tracer-slowed host in the loop).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
if [ "${1:-tests}" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -60 gpurun_out/t.log; exit 1; }
  tail -3 gpurun_out/t.log
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -30 gpurun_out/b.log; exit 1; }
tail -1 gpurun_out/b.log | cut -c1-600
TAG=${2:-go}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
python tools/trace_step.py gpurun_out/prof_$TAG 40 --phases --gapstats > gpurun_out/step_$TAG.txt 2>&1 || true
python tools/timeline.py gpurun_out/prof_$TAG --step -2 --min-us 8 > gpurun_out/timeline_$TAG.txt 2>&1 || true
rm -f gpurun_out/prof_$TAG/run_kernel_trace.csv.gz
head -4 gpurun_out/step_$TAG.txt
head -3 gpurun_out/timeline_$TAG.txt
