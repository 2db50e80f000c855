#!/bin/bash
# GN: a coarsest level of up to 2048 cells (one V-cycle level less at 640x480 and 320x240) with 12
# or 24 sweeps, against the product (1024 cells, 12 sweeps): PCG counts and time per iteration
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for v in prod=optical-flow-optimal-transport_amd/foto/libfoto.so c2048s12=abl/libfoto_c2048_12.so c2048s24=abl/libfoto_c2048_24.so; do
  n=${v%%=*}; lib=${v#*=}
  echo "== $n"
  FOTO_LIB=$PWD/$lib FOTO_LIB_LAX=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread \
      -k "gn or GN or classical" tests/test_gpu_parity.py tests/test_gpu_configs.py > gpurun_out/r05_gnc_tests_$n.log 2>&1 || { tail -20 gpurun_out/r05_gnc_tests_$n.log; exit 2; }
  tail -1 gpurun_out/r05_gnc_tests_$n.log
  FOTO_LIB=$PWD/$lib FOTO_LIB_LAX=1 timeout -k 10 120 python tools/gn_time.py 640 480 584 388 320 240 2>&1 | grep "plan:" || exit 3
done
