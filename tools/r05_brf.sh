#!/bin/bash
# k_prox_rhs with branch-free phi / own-mu loads (FOTO_PR_BRFREE=1 build) against the product:
# bit identity (single shard; 3 virtual ranks for the EDGE form), same-box A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
N=$PWD/optical-flow-optimal-transport_amd/foto/libfoto.so; B=$PWD/abl/libfoto_brf.so
FOTO_LIB=$N timeout -k 10 120 python tools/bitcmp.py save /tmp/b_ref.npz || exit 2
FOTO_LIB=$B FOTO_LIB_LAX=1 timeout -k 10 120 python tools/bitcmp.py save /tmp/b_new.npz || exit 2
python tools/bitcmp.py cmp /tmp/b_ref.npz /tmp/b_new.npz || exit 3
FOTO_LIB=$N timeout -k 10 120 python tools/bitcmp.py save /tmp/b_ref3.npz 32 584 388 4 3 || exit 2
FOTO_LIB=$B FOTO_LIB_LAX=1 timeout -k 10 120 python tools/bitcmp.py save /tmp/b_new3.npz 32 584 388 4 3 || exit 2
python tools/bitcmp.py cmp /tmp/b_ref3.npz /tmp/b_new3.npz || exit 3
for rep in 1 2 3; do
  for v in prod brf; do
    if [ $v = prod ]; then L=$N; else L=$B; fi
    FOTO_LIB=$L FOTO_LIB_LAX=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-gn --no-stencil --steps 100 > $O/ab_brf_${v}_$rep.json 2> $O/ab_brf_${v}_$rep.err || { tail -5 $O/ab_brf_${v}_$rep.err; exit 4; }
    echo -n "$v r$rep "; python tools/show_bench.py $O/ab_brf_${v}_$rep.json
  done
done
