#!/bin/bash
# LM-head dX on 256x192 tiles, one K slice per XCD: parity, then interleaved C2 A/B against the previous library
# (xlib/lib_old.so), plus the dX launch's in-step duration (bench --probe 2)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_ops.py -x -q --timeout 240 --timeout-method thread -k "lm_head or c2 or small or gemm" > gpurun_out/lm_tests.log 2>&1 || { tail -40 gpurun_out/lm_tests.log; exit 1; }
tail -2 gpurun_out/lm_tests.log
run() { tag=$1; shift; env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only $BA > gpurun_out/lm_$tag.json 2> gpurun_out/lm_$tag.err || { tail -20 gpurun_out/lm_$tag.err; exit 1; }; python -c "import json;d=json.loads(open('gpurun_out/lm_$tag.json').read().strip().splitlines()[-1]);print('$tag',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"; }
BA="--probe 2" run p_old ERGM_LIB_PATH=xlib/lib_old.so
BA="--probe 2" run p_new ERGM_NONE=1
for i in 1 2 3; do
BA= run old_$i ERGM_LIB_PATH=xlib/lib_old.so
BA= run new_$i ERGM_NONE=1
done
# kernel stats of the new library's step
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lm_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-only > gpurun_out/lm_prof.log 2>&1
python tools/prof_summary.py gpurun_out/lm_prof 0 45 > gpurun_out/lm_summary.txt
head -30 gpurun_out/lm_summary.txt
