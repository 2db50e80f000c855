#!/bin/bash
# GN persistent tail: polls without s_sleep (abl/libfoto_pt0.so) traced
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
FOTO_LIB=$PWD/abl/libfoto_pt0.so FOTO_LIB_LAX=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -k "round5_forms" tests/test_gpu_parity.py > gpurun_out/r05_gn4_tests.log 2>&1 || { tail -30 gpurun_out/r05_gn4_tests.log; exit 2; }
tail -1 gpurun_out/r05_gn4_tests.log
FOTO_LIB=$PWD/abl/libfoto_pt0.so FOTO_LIB_LAX=1 bash tools/r05_gn.sh gn4 || exit 3
