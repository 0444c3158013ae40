set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/host_profile_dp.py 8 > gpurun_out/host_prof_dp8.txt 2>&1 || { tail -20 gpurun_out/host_prof_dp8.txt; exit 1; }
grep -A50 "==== backward" gpurun_out/host_prof_dp8.txt | head -70
AB_ENV_A=ERGM_BWD_CHAINS=1 AB_ENV_B=ERGM_BWD_CHAINS=2 AB_CONFIGS="" bash tools/ab_env.sh && cat gpurun_out/ab_env.txt
