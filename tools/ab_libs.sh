# A/B of two builds of the same sources: $AB_LIB (default ab/lib_old.so, built from the other variant and
# copied there) against the in-tree library, interleaved runs of bench.py (C2 x3, C5 x2) -> gpurun_out/ab.txt
run() { tag=$1; shift; env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab_$tag.json 2>/dev/null || exit 1; echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/ab_$tag.json'));print(d['value'],d['ms_per_step'])")" >> gpurun_out/ab.txt; }
rm -f gpurun_out/ab.txt
for i in 1 2 3; do run old$i ERGM_LIB_PATH=${AB_LIB:-ab/lib_old.so}; run new$i ERGM_NONE=1; done
BENCH_ARGS="--config c5"
for i in 1 2; do run c5old$i ERGM_LIB_PATH=${AB_LIB:-ab/lib_old.so}; run c5new$i ERGM_NONE=1; done
