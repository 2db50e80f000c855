#!/bin/bash
# GN product after the round-5 changes: parity tests, then the traced 640x480 solve
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -k "gn or GN or classical" \
    tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_batch.py tests/test_gpu_bench.py > gpurun_out/r05_gn2_tests.log 2>&1 || { tail -30 gpurun_out/r05_gn2_tests.log; exit 2; }
tail -2 gpurun_out/r05_gn2_tests.log
bash tools/r05_gn.sh gn2 || exit 3
