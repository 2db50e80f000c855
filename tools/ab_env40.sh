#!/bin/bash
# same-box A/B of environment settings, 40 steps, 3 interleaved reps: tools/ab_env40.sh "A=1" "A=0"
for rep in 1 2 3; do
  for setting in "$@"; do
    env $setting timeout -k 10 120 python bench.py --no-cpu-baseline --no-stencil --no-gn --steps 40 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']
print('$setting', d['value'], d['ms_per_step'], {n: round(v['avg_us'],1) for n,v in k.items()})" || exit 1
  done
done
