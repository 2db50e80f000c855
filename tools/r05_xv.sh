#!/bin/bash
# x^ with four elements per lane (FOTO_GQ_XV): bit-identity tests, same-box A/B on the default
# bench, a kernel trace of the default
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gauss.py -k "xhat_four or tfuse" \
    > gpurun_out/r05_xv_tests.log 2>&1 || { tail -30 gpurun_out/r05_xv_tests.log; exit 2; }
tail -1 gpurun_out/r05_xv_tests.log
bash tools/r05_ab.sh xv "FOTO_GQ_XV=0" "FOTO_GQ_XV=1" 3 || exit 3
bash tools/r05_prof.sh xv "FOTO_GQ_XV=1" || exit 5
