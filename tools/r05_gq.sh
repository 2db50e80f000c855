#!/bin/bash
# round 5 Gauss-chain check: the mode-3 tests, a kernel-trace profile of the default bench (the
# gq kernels' durations and the gaps between them) and an A/B of the node kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gauss.py \
    tests/test_gpu_pipe.py tests/test_gpu_parity.py > gpurun_out/r05_gq_tests.log 2>&1 || { tail -30 gpurun_out/r05_gq_tests.log; exit 3; }
tail -3 gpurun_out/r05_gq_tests.log
bash tools/r05_prof.sh gqw "" || exit 4
bash tools/r05_prof.sh gqt "FOTO_GQ_NODES=thread" || exit 4
for t in gqw gqt; do python3 tools/trace_summary.py gpurun_out/prof_$t | grep -E "==|gq_|gaps" ; done > gpurun_out/r05_gq_trace.txt
cat gpurun_out/r05_gq_trace.txt
