#!/bin/bash
# y-axis FFT pass with 8 lines per block (FOTO_FFT_LPB_MAX=8: 64-B row segments, four blocks per CU)
# against 16 (128-B rows, two blocks per CU): same-box A/B of the library builds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
N=$PWD/optical-flow-optimal-transport_amd/foto/libfoto.so
for rep in 1 2 3; do
  for v in prod lpb8; do
    if [ $v = prod ]; then L=$N; else L=$PWD/abl/libfoto_$v.so; fi
    FOTO_LIB=$L FOTO_LIB_LAX=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-gn --no-stencil --steps 100 > $O/ab_lpb_${v}_$rep.json 2> $O/ab_lpb_${v}_$rep.err || { tail -5 $O/ab_lpb_${v}_$rep.err; exit 4; }
    echo -n "$v r$rep "; python tools/show_bench.py $O/ab_lpb_${v}_$rep.json
  done
done
