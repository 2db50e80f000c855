#!/bin/bash
# histogram batch shape (FOTO_GQ_PE voxels per lane per batch x FOTO_GQ_PB batches per chunk):
# same-box A/B of library builds on the default bench, with the hist kernel's time
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
for rep in 1 2; do
  for v in prod pe8pb4 pe8pb2 pe4pb8; do
    if [ $v = prod ]; then L=$PWD/optical-flow-optimal-transport_amd/foto/libfoto.so; else L=$PWD/abl/libfoto_$v.so; fi
    FOTO_LIB=$L FOTO_LIB_LAX=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-gn --no-stencil --steps 100 > $O/ab_hist_${v}_$rep.json 2> $O/ab_hist_${v}_$rep.err || { tail -5 $O/ab_hist_${v}_$rep.err; exit 3; }
    echo -n "$v r$rep "; python tools/show_bench.py $O/ab_hist_${v}_$rep.json
  done
done
for v in pe8pb4 pe8pb2; do
  rm -rf $O/prof_hist_$v
  FOTO_LIB=$PWD/abl/libfoto_$v.so FOTO_LIB_LAX=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_hist_$v -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stencil --no-gn --no-kernel-timing > $O/prof_hist_$v.log 2>&1 || exit 5
  echo "$v: $(grep -h k_gq_hist_perm $O/prof_hist_$v/run_kernel_stats.csv | cut -d, -f1-5)"
done
