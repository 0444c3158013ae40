#!/bin/bash
# Same-box A/B of this tree against another checkout built in-tree (default _ab_old: a git worktree of
# an earlier commit): tools/ab_tree.sh [dir] [bench args...]; two interleaved rounds.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OLD=${1:-_ab_old}
shift || true
for rep in 1 2; do
  for t in new old; do
    d=.; [ $t = old ] && d=$OLD
    (cd $d && timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $GRAFT_REPO_ROOT/gpurun_out/abt_${t}_$rep.log 2>&1) || { tail -20 gpurun_out/abt_${t}_$rep.log; exit 1; }
    python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], r['value'], r['ms_per_step'], r['roofline']['frac'])" gpurun_out/abt_${t}_$rep.log $t
  done
done
