#!/bin/bash
# GN at 640x480: solve times and a kernel trace split by PCG-iteration position
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-gn}
timeout -k 10 120 python tools/gn_time.py 640 480 > gpurun_out/r05_${tag}_time.txt 2>&1 || exit 2
rm -rf gpurun_out/prof_$tag
timeout -k 10 180 rocprofv3 --kernel-trace -f csv -d gpurun_out/prof_$tag -o run -- python3 tools/gn_time.py 640 480 > gpurun_out/prof_$tag.log 2>&1 || exit 3
python3 tools/gn_trace.py gpurun_out/prof_$tag > gpurun_out/r05_${tag}_trace.txt
cat gpurun_out/r05_${tag}_time.txt gpurun_out/r05_${tag}_trace.txt
