#!/bin/bash
# Shifted weight-gradient pairing (ERGM_DW_SHIFT=1): model / train / DP tests under it, then an interleaved A/B.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ERGM_DW_SHIFT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_train.py tests/test_dist_gpu.py tests/test_gpu_dropout.py -x -q --timeout 180 --timeout-method thread > gpurun_out/t_shift.log 2>&1 || { tail -40 gpurun_out/t_shift.log; exit 1; }
tail -2 gpurun_out/t_shift.log
AB_CONFIGS="c4" AB_ENV_A="ERGM_DW_SHIFT=0" AB_ENV_B="ERGM_DW_SHIFT=1" bash tools/ab_env.sh
cat gpurun_out/ab_env.txt
