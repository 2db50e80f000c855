#!/bin/bash
# Same-box A/B of environment switches on the default bench: tools/ab_env.sh "A=1" "A=0" ...
# (each setting run 3 times, interleaved; prints value and the spec/prox/dct kernel averages)
for rep in 1 2 3; do
  for setting in "$@"; do
    env $setting python bench.py --no-cpu-baseline --no-stencil --no-gn --steps 10 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']
print('$setting', d['value'], {n: round(v['avg_us'],1) for n,v in k.items()})"
  done
done
