#!/bin/bash
# Config 5 stand-in on one GPU: the 8-sequence batch through run.py with 1, 2, 3 and 4 workers
# sharing GPU 0 (run.py --devices), twice each; tables + JSON under gpurun_out/
set -o pipefail
O=gpurun_out; mkdir -p $O
for rep in 1 2; do
  for w in ${WORKERS:-1 2 3 4}; do
    devs=$(python3 -c "print(','.join(['0']*$w))")
    timeout -k 10 300 python tools/batch_bench.py --seqs ${SEQS:-8} --gpus $w --devices $devs --out /tmp/c5_${w}_$rep \
        --table $O/c5_s${SEQS:-8}_w${w}_r$rep.md --json $O/c5_s${SEQS:-8}_w${w}_r$rep.json > $O/c5_s${SEQS:-8}_w${w}_r$rep.log 2>&1 || { echo "w=$w failed"; tail -20 $O/c5_s${SEQS:-8}_w${w}_r$rep.log; exit 3; }
    python3 -c "import json; d=json.load(open('$O/c5_s${SEQS:-8}_w${w}_r$rep.json')); print('workers $w rep $rep:', {k: d[k] for k in ('wall_s','loop_s','solve_s','sequences_per_s','loop_over_solve','startup_s')})"
  done
done
