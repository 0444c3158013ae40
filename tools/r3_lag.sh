#!/bin/bash
# Forward chain lag (ERGM_FWD_LAG): chain 2 enqueued k launches behind chain 1; C2, 2 interleaved rounds.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 180 --timeout-method thread -k "full_c2 or chains" > gpurun_out/t_lag.log 2>&1 || { tail -30 gpurun_out/t_lag.log; exit 1; }
ERGM_FWD_LAG=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 180 --timeout-method thread -k "full_c2 or chains" >> gpurun_out/t_lag.log 2>&1 || { tail -30 gpurun_out/t_lag.log; exit 1; }
grep passed gpurun_out/t_lag.log
run() { tag=$1; shift; env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/lag_$tag.json 2>/dev/null || { echo "$tag FAILED"; return; }; echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/lag_$tag.json'));print(d['value'],d['ms_per_step'])")"; }
for r in 1 2; do for k in 0 1 3 5 8; do run k${k}_$r ERGM_FWD_LAG=$k; done; done
