#!/bin/bash
# Same-box comparison of several in-tree checkouts (git worktrees built in place) on one bench config:
#   tools/bisect_c4.sh "<dir>:<bench args>" ...   (two interleaved rounds; dir "." = this tree)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in "$@"; do
    d=${v%%:*}; a=${v#*:}
    (cd $d && timeout -k 10 300 python bench.py $a > $GRAFT_REPO_ROOT/gpurun_out/bis.log 2>&1) || { tail -5 gpurun_out/bis.log; exit 1; }
    python -c "import json,sys; r=json.loads(open('gpurun_out/bis.log').read().strip().splitlines()[-1]); print(sys.argv[1], r['value'], r['ms_per_step'])" $d
  done
done
