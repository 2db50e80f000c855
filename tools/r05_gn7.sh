#!/bin/bash
# GN level kernels at four blocks per CU (level-0 B loaded after stage 1, r in f's LDS space):
# GN tests, timing against the previous build (abl/libfoto_gnold.so), kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -k "gn or GN or classical" \
    tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_batch.py tests/test_dropin.py > gpurun_out/r05_gn7_tests.log 2>&1 || { tail -30 gpurun_out/r05_gn7_tests.log; exit 3; }
tail -1 gpurun_out/r05_gn7_tests.log
for r in 1 2; do
  for v in new old; do
    echo "== $v rep $r"
    if [ $v = old ]; then L=$PWD/abl/libfoto_gnold.so; else L=$PWD/optical-flow-optimal-transport_amd/foto/libfoto.so; fi
    FOTO_LIB=$L timeout -k 10 120 python tools/gn_time.py 640 480 320 240 584 388 2>&1 | grep "plan:" || exit 4
  done
done
bash tools/r05_gn.sh gn7 || exit 5
