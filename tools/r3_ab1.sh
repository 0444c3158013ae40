# In-step A/B: per-block vs stacked caption K/V gradients, and the KS2 backward overrides
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OV="3073,768,2048,1,1,37,1 769,3072,2048,1,1,37,1 769,768,2048,1,1,34,1 769,2304,2048,1,1,33,1 2048,768,3072,0,0,33,1 2048,768,2304,0,0,33,1 2048,768,768,0,0,35,1"
one() {  # tag, env..., [-- overrides]
  tag=$1; shift
  if [ "$1" = "OV" ]; then shift; env "$@" timeout -k 10 200 python tools/bench_override.py $OV -- --no-cpu-baseline --no-gpu-only > gpurun_out/ab1.log 2>&1 || { tail -5 gpurun_out/ab1.log; exit 1; }
  else env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/ab1.log 2>&1 || { tail -5 gpurun_out/ab1.log; exit 1; }; fi
  python -c "import json,sys; r=json.loads(open('gpurun_out/ab1.log').read().strip().splitlines()[-1]); print(sys.argv[1], r['value'], r['ms_per_step'], r['roofline']['achieved'], flush=True)" $tag | tee -a gpurun_out/r3_ab1.txt
}
rm -f gpurun_out/r3_ab1.txt
for rep in 1 2 3; do
  one split ERGM_CAPKV_SPLIT=1
  one stacked ERGM_CAPKV_SPLIT=0
  one split+ov OV ERGM_CAPKV_SPLIT=1
  one stacked+ov OV ERGM_CAPKV_SPLIT=0
done
