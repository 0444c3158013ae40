#!/bin/bash
# Bound fork points (ERGM_BIND_FORKS): model / dropout / dist GPU tests, then an interleaved C2 A/B and the
# GPU-only kernel trace of the new default.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_dropout.py tests/test_dist_gpu.py tests/test_gpu_train.py -x -q --timeout 180 --timeout-method thread > gpurun_out/t_bind.log 2>&1 || { tail -40 gpurun_out/t_bind.log; exit 1; }
tail -2 gpurun_out/t_bind.log
AB_CONFIGS="c4" AB_ENV_A="ERGM_BIND_FORKS=0" AB_ENV_B="ERGM_BIND_FORKS=1" bash tools/ab_env.sh
cat gpurun_out/ab_env.txt
bash tools/r3_check.sh notests bind1 | tail -3
