#!/bin/bash
# Config-5 kernel statistics: MX-fp8 forward GEMMs vs bf16, rocprofv3 kernel trace of a short bench.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for m in mx bf16; do
  a=""; [ $m = bf16 ] && a="--no-fp8"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof_$m -o run -- python3 bench.py --config c5 --no-cpu-baseline --no-gpu-only --steps 10 --warmup 3 $a > gpurun_out/c5prof_$m.json 2> gpurun_out/c5prof_$m.err
done
find gpurun_out/c5prof_mx gpurun_out/c5prof_bf16 -name '*kernel_stats.csv' | sort
