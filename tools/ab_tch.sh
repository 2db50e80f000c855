#!/bin/bash
# k_prox_rhs planes per chunk (FOTO_PR_TCH) sweep on the default bench, interleaved twice:
# tools/ab_tch.sh 8 11 16 ...
for rep in 1 2; do
  for t in "$@"; do
    FOTO_PR_TCH=$t timeout -k 10 120 python bench.py --no-cpu-baseline --no-stencil --no-gn --steps 10 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('TCH=$t', d['value'], round(d['kernels']['prox']['avg_us'],1))" || exit $?
  done
done
