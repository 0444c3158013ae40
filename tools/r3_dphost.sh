# DP host cost under a fake 8-rank process group: bench line + cProfile of the host work
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ERGM_BENCH_FAKE_PG=8 timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/r3_fakepg.json 2> gpurun_out/r3_fakepg.err || { tail -20 gpurun_out/r3_fakepg.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r3_fakepg.json').read().strip().splitlines()[-1]);print({k:d.get(k) for k in ('value','ms_per_step','host_enqueue_ms_per_step','host_busy_ms_per_step_in_timed_loop','host_enqueue_ms_per_step_in_timed_loop')})"
timeout -k 10 200 python tools/host_profile_dp.py 8 > gpurun_out/r3_dpprof.txt 2>&1 || { tail -20 gpurun_out/r3_dpprof.txt; exit 1; }
grep -A 45 "Ordered by" gpurun_out/r3_dpprof.txt | head -50
