cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/host_profile_dp.py 8 > gpurun_out/r3_hostprof8.txt 2>&1 || { tail -20 gpurun_out/r3_hostprof8.txt; exit 1; }
timeout -k 10 200 python tools/host_profile_dp.py 1 > gpurun_out/r3_hostprof1.txt 2>&1 || { tail -20 gpurun_out/r3_hostprof1.txt; exit 1; }
head -60 gpurun_out/r3_hostprof8.txt
