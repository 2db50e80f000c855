#!/bin/bash
# GN LDS-resident last level + coarsest (k_mg_ltail, default) : bit-identity, GN tests, traces
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread -k "round5_forms" tests/test_gpu_parity.py \
    > gpurun_out/r05_gn5_tests.log 2>&1 || { tail -40 gpurun_out/r05_gn5_tests.log; exit 2; }
grep -E "PCG its|passed|failed" gpurun_out/r05_gn5_tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -k "gn or GN or classical" \
    tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_batch.py tests/test_dropin.py > gpurun_out/r05_gn5_tests2.log 2>&1 || { tail -30 gpurun_out/r05_gn5_tests2.log; exit 3; }
tail -1 gpurun_out/r05_gn5_tests2.log
bash tools/r05_gn.sh gn5 || exit 4
FOTO_MG_LTAIL=0 bash tools/r05_gn.sh gn5sep || exit 5
timeout -k 10 120 python tools/gn_time.py 584 388 320 240 160 120 2>&1 | grep "plan:" || exit 6
