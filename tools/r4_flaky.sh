#!/bin/bash
# is the fused-optimizer mismatch at (2, 64, 256) deterministic?  three passes of the fused-optimizer and fused-attention
# bitwise tests, plus the same test with the fused attention backward off
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -q --timeout 240 --timeout-method thread -k "fused_optimizer or fused_attention or deterministic" > gpurun_out/fl_$i.log 2>&1; echo "pass $i rc=$?"; grep -E "passed|failed|FAILED" gpurun_out/fl_$i.log | tail -4
done
ERGM_ATTN_FUSE=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -q --timeout 240 --timeout-method thread -k "fused_optimizer" > gpurun_out/fl_noaf.log 2>&1; echo "noaf rc=$?"; grep -E "passed|failed|FAILED" gpurun_out/fl_noaf.log | tail -4
ERGM_XQ_FUSE=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -q --timeout 240 --timeout-method thread -k "fused_optimizer" > gpurun_out/fl_noxq.log 2>&1; echo "noxq rc=$?"; grep -E "passed|failed|FAILED" gpurun_out/fl_noxq.log | tail -4
exit 0
