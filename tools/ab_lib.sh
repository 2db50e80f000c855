#!/bin/bash
# interleaved A/B of the prefetch depth builds
B="python bench.py --no-cpu-baseline --no-gn --no-stencil --steps 20"
for rep in 1 2; do
  for v in pf3:optical-flow-optimal-transport_amd/foto/libfoto.so pf0:build_ab/libfoto_pf0.so pf6:build_ab/libfoto_pf6.so; do
    n=${v%%:*}; lib=${v#*:}
    FOTO_LIB=$PWD/$lib timeout -k 10 120 $B > gpurun_out/ab_$n.log 2>&1 || exit $?
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_$n.log').read().strip().split('\n')[-1]);print('$n',d['value'],d['roofline']['avg_launch_us'],d['cg_iters_per_step'])"
  done
done
