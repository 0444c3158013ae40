# In-step A/B of stream priorities (update stream low / weight-gradient stream high)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
python -c "import torch; print('priority range (least, greatest):', torch.cuda.Stream.priority_range())"
one() { tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-gpu-only > gpurun_out/prio.log 2>&1 || { tail -5 gpurun_out/prio.log; exit 1; }
  python -c "import json,sys; r=json.loads(open('gpurun_out/prio.log').read().strip().splitlines()[-1]); print(sys.argv[1], r['value'], r['ms_per_step'], r['roofline']['achieved'], flush=True)" $tag | tee -a gpurun_out/r3_prio.txt
}
rm -f gpurun_out/r3_prio.txt
for rep in 1 2 3; do
  one base X=0
  one opt_low ERGM_OPT_PRIORITY=${LOW:-1}
  one side_high ERGM_SIDE_PRIORITY=${HIGH:--1}
  one both ERGM_OPT_PRIORITY=${LOW:-1} ERGM_SIDE_PRIORITY=${HIGH:--1}
done
