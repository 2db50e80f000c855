#!/bin/bash
# GN: parity tests of the product and of abl/libfoto_pf.so, then traced 640x480 solves: product
# (folded update), FOTO_GN_FOLD=0 (k_gnp_upd), and the up-front-load level kernels (pf)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T="tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_batch.py"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -k "gn or GN or classical" $T \
    > gpurun_out/r05_gn_tests.log 2>&1 || { tail -30 gpurun_out/r05_gn_tests.log; exit 2; }
tail -2 gpurun_out/r05_gn_tests.log
FOTO_LIB=$PWD/abl/libfoto_pf.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    -k "gn or GN or classical" $T > gpurun_out/r05_gn_tests_pf.log 2>&1 || { tail -30 gpurun_out/r05_gn_tests_pf.log; exit 3; }
tail -2 gpurun_out/r05_gn_tests_pf.log
bash tools/r05_gn.sh gnfold || exit 4
FOTO_GN_FOLD=0 bash tools/r05_gn.sh gnsep || exit 5
FOTO_LIB=$PWD/abl/libfoto_pf.so bash tools/r05_gn.sh gnpf || exit 6
