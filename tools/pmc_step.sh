#!/bin/bash
# In-step PMC passes of the C2 bench (one counter group per run): what the kernel classes wait on when they
# share the chip.  tools/pmc_step.sh -> gpurun_out/pmcs_<i>/ and a per-class summary (tools/pmc_step_sum.py)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for ctr in "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE" "TD_TD_BUSY TD_TC_STALL" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/pmcs_$i -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gpu-only > gpurun_out/pmcs_$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/pmcs_$i.log; exit 1; }
done
python3 tools/pmc_step_sum.py gpurun_out/pmcs_ $i
