#!/bin/bash
# Iteration check on the GPU box: GPU test suite (optionally a -k filter), then a short C2 bench.
#   tools/gpu_check.sh [pytest -k expression] [bench args...]
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
K=${1:-}
shift || true
if [ -n "$K" ] && [ "$K" != "all" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -k "$K" > gpurun_out/t.log 2>&1 || { tail -60 gpurun_out/t.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -60 gpurun_out/t.log; exit 1; }
fi
tail -5 gpurun_out/t.log
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/b.log 2>&1 || { tail -30 gpurun_out/b.log; exit 1; }
tail -1 gpurun_out/b.log
