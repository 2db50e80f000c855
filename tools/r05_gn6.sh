#!/bin/bash
# GN graph of 4 iterations (default) vs 2: GN tests, timing both ways
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -k "gn or GN or classical" \
    tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_batch.py tests/test_dropin.py > gpurun_out/r05_gn6_tests.log 2>&1 || { tail -30 gpurun_out/r05_gn6_tests.log; exit 3; }
tail -1 gpurun_out/r05_gn6_tests.log
for r in 1 2; do
  for g in 4 2; do
    echo "== FOTO_GN_GRAPH=$g rep $r"
    FOTO_GN_GRAPH=$g timeout -k 10 120 python tools/gn_time.py 640 480 320 240 2>&1 | grep "plan:" || exit 4
  done
done
bash tools/r05_gn.sh gn6 || exit 5
