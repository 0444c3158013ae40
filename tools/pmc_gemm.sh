#!/bin/bash
# PMC passes (one counter group per run) over one isolated GEMM configuration (tools/gemm_one.py):
#   tools/pmc_gemm.sh TAG CFG LAYOUT M N K   -> gpurun_out/pmcg_TAG_<pass>/ and a summary (tools/pmc_gemm_sum.py)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=$1; shift
i=0
for ctr in "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE" "TA_DATA_STALLED_BY_TC_CYCLES TA_BUSY" \
           "TD_TD_BUSY TD_TC_STALL" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS" \
           "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr -d gpurun_out/pmcg_${TAG}_$i -o run --output-format csv -- python3 tools/gemm_one.py "$@" 200 > gpurun_out/pmcg_${TAG}_$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/pmcg_${TAG}_$i.log; exit 1; }
done
python3 tools/pmc_gemm_sum.py gpurun_out/pmcg_${TAG}_ $i
