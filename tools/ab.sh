#!/bin/bash
# One same-box A/B driver for every switch (replaces round 5's single-use tools/r05_*.sh):
#   tools/ab.sh TAG [-r REPS] [-t "PYTEST ARGS"] [-b "BENCH ARGS"] VARIANT [VARIANT ...]
# VARIANT is  name=ENV1=v1,ENV2=v2   (environment switches; "name=" for the defaults)
#         or  name=lib:path/to/libfoto.so   (a library build, loaded through FOTO_LIB)
# -t: the given pytest selection runs once per variant first (parity before timing; a failure
#     stops the script); then REPS interleaved bench runs per variant (default 2), each line's
#     value, prox launch time and fraction printed; lines under gpurun_out/ab_TAG_NAME_REP.json.
# Run from the repo root on the GPU box.
set -o pipefail
tag=$1; shift
reps=2; tests=""; bargs="--no-cpu-baseline --no-gn --no-stencil --steps 100"
while getopts "r:t:b:" o; do
  case $o in r) reps=$OPTARG ;; t) tests=$OPTARG ;; b) bargs=$OPTARG ;; *) exit 2 ;; esac
done
shift $((OPTIND - 1))
O=gpurun_out; mkdir -p $O
venv() {   # the environment of a variant, one assignment per line
  local spec=${1#*=}
  if [[ $spec == lib:* ]]; then echo "FOTO_LIB=$PWD/${spec#lib:}"; echo "FOTO_LIB_LAX=1"
  elif [ -n "$spec" ]; then echo "$spec" | tr ',' '\n'; fi
}
run_env() { local v=$1; shift; local e=(); while read -r kv; do [ -n "$kv" ] && e+=("$kv"); done < <(venv "$v"); env "${e[@]}" "$@"; }
if [ -n "$tests" ]; then
  for v in "$@"; do
    n=${v%%=*}
    run_env "$v" timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread $tests \
      > $O/ab_${tag}_${n}_tests.log 2>&1 || { echo "tests $n failed"; tail -20 $O/ab_${tag}_${n}_tests.log; exit 3; }
    echo "tests $n: $(tail -1 $O/ab_${tag}_${n}_tests.log)"
  done
fi
for r in $(seq 1 $reps); do
  for v in "$@"; do
    n=${v%%=*}; f=$O/ab_${tag}_${n}_$r
    run_env "$v" timeout -k 10 300 python bench.py $bargs > $f.json 2> $f.err || { echo "bench $n/$r failed"; tail -5 $f.err; exit 4; }
    python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d.get('roofline') or {}
ev = r.get('event_bracketed') or r
print(f\"{sys.argv[2]:>12s} rep {sys.argv[3]}: {d['value']:9.2f} it/s  prox {ev.get('avg_launch_us')} us  frac {ev.get('frac')}\")" $f.json $n $r
  done
done
