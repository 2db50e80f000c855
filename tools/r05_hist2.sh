#!/bin/bash
# the 8 x 4 histogram batches against the 16 x 2 build: bit identity (one shard at the bench grid,
# 3 virtual ranks at 584x388x32), the Gauss tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
N=$PWD/optical-flow-optimal-transport_amd/foto/libfoto.so; P=$PWD/abl/libfoto_pe16pb2.so
FOTO_LIB=$N timeout -k 10 120 python tools/bitcmp.py save $O/h_new.npz || exit 2
FOTO_LIB=$P FOTO_LIB_LAX=1 timeout -k 10 120 python tools/bitcmp.py save $O/h_old.npz || exit 2
python tools/bitcmp.py cmp $O/h_new.npz $O/h_old.npz || exit 3
FOTO_LIB=$N timeout -k 10 120 python tools/bitcmp.py save $O/h_new3.npz 32 584 388 4 3 || exit 2
FOTO_LIB=$P FOTO_LIB_LAX=1 timeout -k 10 120 python tools/bitcmp.py save $O/h_old3.npz 32 584 388 4 3 || exit 2
python tools/bitcmp.py cmp $O/h_new3.npz $O/h_old3.npz || exit 3
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gauss.py > $O/h_tests.log 2>&1 || { tail -20 $O/h_tests.log; exit 4; }
tail -1 $O/h_tests.log
