#!/bin/bash
# Config-5 kernel statistics: rocprofv3 kernel trace of a short bench per variant (args: tag=ENV=VAL ... or tag=bf16).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for spec in "$@"; do
  tag=${spec%%=*}; ev=${spec#*=}
  a=""; [ "$ev" = bf16 ] && { a="--no-fp8"; ev="ERGM_NONE=1"; }
  env $ev timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/c5prof_$tag -o run -- python3 bench.py --config c5 --no-cpu-baseline --no-gpu-only --steps 10 --warmup 3 $a > gpurun_out/c5prof_$tag.json 2> gpurun_out/c5prof_$tag.err
done
