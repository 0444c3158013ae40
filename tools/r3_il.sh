set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "every_pipelined or bias_grad" > gpurun_out/r3_il_tests.log 2>&1 || { tail -30 gpurun_out/r3_il_tests.log; exit 1; }
tail -2 gpurun_out/r3_il_tests.log
timeout -k 10 600 python tools/gemm_tune.py --cfgs 0,25,2,26,3,27,6,28,8,29,10,30,14,31,1,32 > gpurun_out/r3_il_tune.txt 2>&1
tail -25 gpurun_out/r3_il_tune.txt
