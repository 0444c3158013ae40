#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/concurrency_probe.py 2>&1 | grep -v amdgpu.ids
