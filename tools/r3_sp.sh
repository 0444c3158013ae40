set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "every_pipelined or bias_grad or layouts" > gpurun_out/r3_sp_tests.log 2>&1 || { tail -30 gpurun_out/r3_sp_tests.log; exit 1; }
tail -2 gpurun_out/r3_sp_tests.log
timeout -k 10 700 python tools/gemm_tune.py --cfgs 0,33,34,35,36,2,37,38,3,39,10,40,8,41,7,42,4,43,5,44 > gpurun_out/r3_sp_tune.txt 2>&1
cp gpurun_out/gemm_tune.json gpurun_out/r3_sp_tune.json
tail -23 gpurun_out/r3_sp_tune.txt
