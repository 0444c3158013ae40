# One gpurun command that regenerates the round's judged measurements (bench lines, kernel trace,
# PMC passes, isolated kernel benches).  Every step runs under its own time limit; the first failure
# ends the script.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py > gpurun_out/m_bench_c2.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/m_bench_c2b.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/m_prof_c2 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-only > gpurun_out/m_prof_c2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/m_pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gpu-only --no-overlap-optim > gpurun_out/m_pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/m_pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gpu-only --no-overlap-optim > gpurun_out/m_pmc_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 -d gpurun_out/m_pmc_mfma -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gpu-only --no-overlap-optim > gpurun_out/m_pmc_mfma.log 2>&1
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > gpurun_out/m_bench_c4.log 2>&1
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/m_bench_c5.log 2>&1
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-fp8 > gpurun_out/m_bench_c5_bf16.log 2>&1
timeout -k 10 120 python tools/op_bench.py > gpurun_out/m_op_bench.log 2>&1
timeout -k 10 120 python tools/attn_bench.py > gpurun_out/m_attn_bench.log 2>&1
