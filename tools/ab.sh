#!/bin/bash
# A/B bench variants in one GPU call: tools/ab.sh "<label>:<env assignments>:<bench args>" ...
# Each variant runs twice (interleaved) to expose box noise.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in "$@"; do
    label=${v%%:*}; rest=${v#*:}; envs=${rest%%:*}; args=${rest#*:}
    env $envs timeout -k 10 300 python bench.py --no-cpu-baseline $args > gpurun_out/ab_${label}_$rep.log 2>&1 || { tail -20 gpurun_out/ab_${label}_$rep.log; exit 1; }
    python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], r['value'], r['ms_per_step'], r['host_enqueue_ms_per_step'])" gpurun_out/ab_${label}_$rep.log $label
  done
done
