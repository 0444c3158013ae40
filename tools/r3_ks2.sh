set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "every_pipelined or bias_grad or layouts or adamw" > gpurun_out/r3_ks2_tests.log 2>&1 || { tail -30 gpurun_out/r3_ks2_tests.log; exit 1; }
tail -2 gpurun_out/r3_ks2_tests.log
timeout -k 10 700 python -u -m pytest tests/test_optim_interchange.py tests/test_dist_gpu.py tests/test_gpu_c5.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r3_newtests.log 2>&1 || { tail -40 gpurun_out/r3_newtests.log; exit 1; }
tail -3 gpurun_out/r3_newtests.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_tail_bench.json 2> gpurun_out/r3_tail_bench.err
python -c "import json;d=json.loads(open('gpurun_out/r3_tail_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['host_enqueue_ms_per_step'],d['train_metrics'])"
timeout -k 10 400 python tools/gemm_tune.py --cfgs 0,33,34,8,35,7,36,2,37 > gpurun_out/r3_ks2_tune.txt 2>&1
cp gpurun_out/gemm_tune.json gpurun_out/r3_ks2_tune.json
tail -22 gpurun_out/r3_ks2_tune.txt
