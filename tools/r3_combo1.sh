cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r3_distgpu.log 2>&1 || { tail -30 gpurun_out/r3_distgpu.log; exit 1; }
tail -2 gpurun_out/r3_distgpu.log
bash tools/r3_dphost.sh || exit 1
bash tools/r3_prio.sh || exit 1
