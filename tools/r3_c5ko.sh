#!/bin/bash
# Config-5 knock-out attribution (ERGM_DIAG_SKIP classes, common.h; results wrong, timing only), MX-fp8 default.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { tag=$1; shift; env "$@" timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline --no-gpu-only --steps 15 > gpurun_out/ko_$tag.json 2>gpurun_out/ko_$tag.err || { echo "$tag FAILED"; tail -3 gpurun_out/ko_$tag.err; exit 1; }; echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/ko_$tag.json'));print(d['ms_per_step'])")"; }
for r in 1 2; do
  run base$r ERGM_NONE=1
  for k in 1024 1 512 8 32 4 2048 128; do run k${k}_$r ERGM_DIAG_SKIP=$k; done
done
