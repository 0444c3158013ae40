#!/bin/bash
# forward / backward+optimizer device time per step (ERGM_BENCH_PHASES), and the forward GEMMs' in-step durations
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ERGM_BENCH_PHASES=gpurun_out/ph_c2.json ERGM_BENCH_FWD_DETAIL=gpurun_out/ph_fwd_detail.json timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/ph_b.json 2> gpurun_out/ph_b.err
cat gpurun_out/ph_c2.json; echo
python - <<'PY'
import json
d = json.load(open("gpurun_out/ph_fwd_detail.json"))
print(len(d), "forward GEMM launches; total us", round(sum(x["us"] for x in d), 1))
for x in d[:14]: print(x)
PY
