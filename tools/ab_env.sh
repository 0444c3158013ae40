# A/B of one environment switch in the same build: interleaved bench.py runs with $AB_ENV_A against
# $AB_ENV_B (e.g. AB_ENV_A=ERGM_LMHEAD_TAIL=0 AB_ENV_B=ERGM_LMHEAD_TAIL=1), C2 x3 then $AB_CONFIGS
# (default "c4 c5") x2 each -> gpurun_out/ab_env.txt
run() { tag=$1; shift; env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/abe_$tag.json 2>/dev/null || exit 1; echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/abe_$tag.json'));print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])")" >> gpurun_out/ab_env.txt; }
rm -f gpurun_out/ab_env.txt
for i in 1 2 3; do run a$i $AB_ENV_A; run b$i $AB_ENV_B; done
for c in ${AB_CONFIGS-c4 c5}; do
  BENCH_ARGS="--config $c"
  for i in 1 2; do run ${c}a$i $AB_ENV_A; run ${c}b$i $AB_ENV_B; done
done
