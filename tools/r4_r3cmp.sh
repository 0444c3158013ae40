#!/bin/bash
# same-box comparison of the round-3 tree (xold/, built from commit a29c3e1) and the current one, C2 / C4 / C5
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { tag=$1; dir=$2; shift; shift; (cd $dir && timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-gpu-only > $GRAFT_REPO_ROOT/gpurun_out/cmp_$tag.json 2> $GRAFT_REPO_ROOT/gpurun_out/cmp_$tag.err) || { tail -20 gpurun_out/cmp_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/cmp_$tag.json').read().strip().splitlines()[-1]);print('$tag',d['value'],d['ms_per_step'])"; }
for i in 1 2; do
run c5_r3_$i xold --config c5
run c5_r4_$i . --config c5
run c4_r3_$i xold --config c4
run c4_r4_$i . --config c4
run c2_r3_$i xold
run c2_r4_$i .
done
