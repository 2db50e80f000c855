#!/bin/bash
# GN PCG kernels' grid (FOTO_GN_GRID blocks per CU: 2 default, 3, 4, 5): GN tests at 4, timing
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
FOTO_GN_GRID=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -k "gn or GN or classical" \
    tests/test_gpu_parity.py tests/test_gpu_configs.py > gpurun_out/r05_gn8_tests.log 2>&1 || { tail -30 gpurun_out/r05_gn8_tests.log; exit 3; }
tail -1 gpurun_out/r05_gn8_tests.log
for r in 1 2; do
  for g in 2 3 4 5; do
    echo "== FOTO_GN_GRID=$g rep $r"
    FOTO_GN_GRID=$g timeout -k 10 120 python tools/gn_time.py 640 480 584 388 2>&1 | grep "plan:" || exit 4
  done
done
