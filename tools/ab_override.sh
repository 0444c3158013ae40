#!/bin/bash
# A/B of GEMM configuration overrides inside the bench step: tools/ab_override.sh "label:M,N,K,al,bl,cfg,split[ ...]" ...
# ("label:" alone = the built-in table); two interleaved rounds.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rep in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    l=${v%%:*}; o=${v#*:}
    if [ -z "$o" ]; then
      timeout -k 10 300 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/ov.log 2>&1 || { tail -5 gpurun_out/ov.log; exit 1; }
    else
      timeout -k 10 300 python tools/bench_override.py $o -- --no-cpu-baseline --no-gpu-only > gpurun_out/ov.log 2>&1 || { tail -5 gpurun_out/ov.log; exit 1; }
    fi
    python -c "import json,sys; r=json.loads(open('gpurun_out/ov.log').read().strip().splitlines()[-1]); print(sys.argv[1], r['value'], r['ms_per_step'])" $l
  done
done
