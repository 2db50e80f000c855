#!/bin/bash
# FETCH_SIZE / WRITE_SIZE (one counter per rocprofv3 pass, as MI355X_MICROARCH.md prescribes) of the
# bench's big kernels under each library build -- the traffic side of a tools/ab.sh comparison.
#   tools/pmc_ab.sh TAG name=lib:path.so ...   (name= for the product library)
# Prints raw KiB per launch; a bytes figure needs the calibration of tools/profile_round.sh.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
O=gpurun_out; mkdir -p $O
args="--steps 3 --warmup 1 --no-cpu-baseline --no-stencil --no-gn --no-kernel-timing"
for v in "$@"; do
  n=${v%%=*}; spec=${v#*=}
  if [[ $spec == lib:* ]]; then export FOTO_LIB=$PWD/${spec#lib:} FOTO_LIB_LAX=1; else unset FOTO_LIB FOTO_LIB_LAX; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$O/pmcab_${tag}_${n}_$c; rm -rf $d
    timeout -s KILL 120 rocprofv3 --pmc $c -f csv -d $d -o run -- python3 bench.py $args > $d.log 2>&1 || { echo "$n $c failed"; tail -5 $d.log; exit 2; }
  done
  python3 - "$O/pmcab_${tag}_${n}" "$n" <<'PY'
import sys
sys.path.insert(0, "tools")
from summarize_profile import pmc
base, name = sys.argv[1], sys.argv[2]
f, _ = pmc(base + "_FETCH_SIZE", "FETCH_SIZE")
w, _ = pmc(base + "_WRITE_SIZE", "WRITE_SIZE")
for k in ("prox", "dct_fft_fwd", "dct_fft_inv", "gq_xhat", "gq_hist"):
    if k in f:
        print(f"{name:>10s} {k:12s} FETCH {f[k] / 1024:9.1f} MiB  WRITE {w.get(k, 0) / 1024:9.1f} MiB per launch (raw)")
PY
done
