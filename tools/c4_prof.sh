#!/bin/bash
# Kernel trace of the C4-size workload (1024x1024x64, one GPU) for profiles/: rocprofv3 --stats
# around tools/size_sweep.py at that size only.  (run from the repo root on the GPU box)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf gpurun_out/prof_c4
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_c4 -o run -- python3 tools/size_sweep.py 1024x1024x64 > gpurun_out/prof_c4.log 2>&1
