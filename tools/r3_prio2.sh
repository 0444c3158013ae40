#!/bin/bash
# Scheduling priority of the critical chains: the caller's stream (data-gradient chain, forward chain 1) and the
# second forward chain high (-1), the weight-gradient / optimizer streams default; C2 x3 + C4 x2 interleaved.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
AB_CONFIGS="c4" AB_ENV_A="ERGM_NONE=1" AB_ENV_B="ERGM_MAIN_PRIO=-1 ERGM_FWD2_PRIO=-1" bash tools/ab_env.sh
cat gpurun_out/ab_env.txt
