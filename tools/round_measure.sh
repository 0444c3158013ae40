#!/bin/bash
# Round-4 judged measurements in one gpurun call (the GPU test suite runs separately: tools/r4_tests.sh): bench lines (C2 default with the CPU
# baseline, C4, C5 MX / per-row fp8 / bf16), the C2 kernel trace + PMC passes, the DP host cost under a fake
# 8-rank group.  Every GPU step has its own time limit; the first failure ends the script.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py > gpurun_out/f4_bench_c2.json 2> gpurun_out/f4_bench_c2.err
tail -c 400 gpurun_out/f4_bench_c2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/f4_prof4_c2 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-only > gpurun_out/f4_prof4_c2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/f4_pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gpu-only --no-overlap-optim > gpurun_out/f4_pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/f4_pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gpu-only --no-overlap-optim > gpurun_out/f4_pmc_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 -d gpurun_out/f4_pmc_mfma -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gpu-only --no-overlap-optim > gpurun_out/f4_pmc_mfma.log 2>&1
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > gpurun_out/f4_bench_c4.json 2> gpurun_out/f4_bench_c4.err
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/f4_bench_c5.json 2> gpurun_out/f4_bench_c5.err
ERGM_FP8_MX=0 timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/f4_bench_c5_row.json 2> gpurun_out/f4_bench_c5_row.err
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-fp8 > gpurun_out/f4_bench_c5_bf16.json 2> gpurun_out/f4_bench_c5_bf16.err
for f in c4 c5 c5_row c5_bf16; do python -c "import json;d=json.loads(open('gpurun_out/f4_bench_$f.json').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'])"; done
ERGM_BENCH_FAKE_PG=8 timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/f4_fakepg.json 2> gpurun_out/f4_fakepg.err
python -c "import json;d=json.loads(open('gpurun_out/f4_fakepg.json').read().strip().splitlines()[-1]);print({k:d.get(k) for k in ('value','ms_per_step','host_enqueue_ms_per_step','host_busy_ms_per_step_in_timed_loop')})"
