#!/bin/bash
# A/B of an env switch on the default bench (no CPU baselines / GN / stencil side lines):
#   tools/r05_ab.sh TAG "ENV_A" "ENV_B" [reps]   (e.g. "FOTO_DCT_XT=1" "FOTO_DCT_XT=0")
set -o pipefail
O=gpurun_out; mkdir -p $O
tag=$1; A=$2; B=$3; reps=${4:-2}
for r in $(seq 1 $reps); do
  for v in A B; do
    e=$([ $v = A ] && echo "$A" || echo "$B")
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --no-gn --no-stencil --steps 100 > $O/ab_${tag}_${v}$r.json 2> $O/ab_${tag}_${v}$r.err || { echo "bench $v$r failed"; tail -5 $O/ab_${tag}_${v}$r.err; exit 4; }
    echo -n "$v$r [$e] "; python tools/show_bench.py $O/ab_${tag}_${v}$r.json
  done
done
