set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_optim_interchange.py tests/test_dist_gpu.py tests/test_gpu_c5.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -k "interchange or reference or nccl or dp2 or c5_bench or full_c2 or full_c4 or overlapped" > gpurun_out/r3_newtests.log 2>&1 || { tail -40 gpurun_out/r3_newtests.log; exit 1; }
tail -3 gpurun_out/r3_newtests.log
ERGM_BENCH_FAKE_PG=8 timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/r3_fakepg8.log 2>&1
python -c "import json; r=json.loads(open('gpurun_out/r3_fakepg8.log').read().strip().splitlines()[-1]); print('fakepg8', r['ms_per_step'], r['host_enqueue_ms_per_step'], r['host_busy_ms_per_step_in_timed_loop'], r['dp'])"
ROUNDS=2 bash tools/ab_override.sh "base:" \
 "il30:1024,3072,768,0,1,30,1 2048,3072,768,0,0,30,1 2048,18432,768,0,1,30,1 1024,2304,768,0,1,27,1" 2>&1 | grep -v amdgpu.ids
