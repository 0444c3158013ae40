set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r3_base_bench.log 2>&1
tail -1 gpurun_out/r3_base_bench.log | cut -c1-400
bash tools/prof_c2.sh r3base > /dev/null 2>&1 || true
python tools/timeline.py gpurun_out/prof_r3base --step 5 --min-us 8 > gpurun_out/r3base_timeline.txt 2>&1 || true
timeout -k 10 300 python tools/gemm_tune.py --auto-only > gpurun_out/r3base_gemm_auto.txt 2>&1
tail -3 gpurun_out/r3base_gemm_auto.txt
