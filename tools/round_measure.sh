#!/bin/bash
# The round's judged measurements in one gpurun call: tools/round_measure.sh TAG [what...]
#   what: bench (C2 line with the CPU baseline), prof (C2 kernel trace + stats), pmc (FETCH / WRITE / MFMA passes),
#         c4, c5 (MX-fp8, per-row fp8, bf16), fakepg (the DP schedule under a fake 8-rank group).  Default: all.
# Outputs gpurun_out/TAG_*.  Every GPU step has its own time limit; the first failure ends the script.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-m}; shift || true
W=${*:-bench prof pmc c4 c5 fakepg}
has() { [[ " $W " == *" $1 "* ]]; }
line() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d['value'],d['ms_per_step'],d.get('roofline',{}).get('frac'),d.get('host_busy_ms_per_step_in_timed_loop'))" $1; }
if has bench; then
  timeout -k 10 300 python bench.py > gpurun_out/${T}_bench_c2.json 2> gpurun_out/${T}_bench_c2.err
  line gpurun_out/${T}_bench_c2.json
fi
if has prof; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c2 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-only > gpurun_out/${T}_prof_c2.log 2>&1
  python tools/prof_summary.py $(dirname $(find gpurun_out/${T}_prof_c2 -name run_kernel_stats.csv | head -1)) 0 40 > gpurun_out/${T}_kernel_stats_summary.txt
  head -25 gpurun_out/${T}_kernel_stats_summary.txt
fi
if has pmc; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${T}_pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gpu-only --no-overlap-optim > gpurun_out/${T}_pmc_fetch.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${T}_pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gpu-only --no-overlap-optim > gpurun_out/${T}_pmc_write.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 -d gpurun_out/${T}_pmc_mfma -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gpu-only --no-overlap-optim > gpurun_out/${T}_pmc_mfma.log 2>&1
  python tools/pmc_traffic.py gpurun_out/${T}_pmc_fetch gpurun_out/${T}_pmc_write gpurun_out/${T}_pmc_traffic.json | tail -5
  python tools/pmc_mfma.py gpurun_out/${T}_pmc_mfma gpurun_out/${T}_pmc_mfma.json | tail -5
fi
if has c4; then
  timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > gpurun_out/${T}_bench_c4.json 2> gpurun_out/${T}_bench_c4.err
  line gpurun_out/${T}_bench_c4.json
fi
if has c5; then
  timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/${T}_bench_c5.json 2> gpurun_out/${T}_bench_c5.err
  ERGM_FP8_MX=0 timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/${T}_bench_c5_row.json 2> gpurun_out/${T}_bench_c5_row.err
  timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-fp8 > gpurun_out/${T}_bench_c5_bf16.json 2> gpurun_out/${T}_bench_c5_bf16.err
  for f in c5 c5_row c5_bf16; do line gpurun_out/${T}_bench_$f.json; done
fi
if has fakepg; then
  ERGM_BENCH_FAKE_PG=8 timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/${T}_fakepg.json 2> gpurun_out/${T}_fakepg.err
  line gpurun_out/${T}_fakepg.json
fi
