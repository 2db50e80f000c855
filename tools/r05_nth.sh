#!/bin/bash
# FFT axis passes at 512 threads per block (FOTO_FFT_NTH_S: strided y / t, FOTO_FFT_NTH_C:
# contiguous x) against 256: bit identity, then a same-box A/B of the library builds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
N=$PWD/optical-flow-optimal-transport_amd/foto/libfoto.so
FOTO_LIB=$N timeout -k 10 120 python tools/bitcmp.py save /tmp/n_ref.npz || exit 2
FOTO_LIB=$PWD/abl/libfoto_nthB.so FOTO_LIB_LAX=1 timeout -k 10 120 python tools/bitcmp.py save /tmp/n_b.npz || exit 2
python tools/bitcmp.py cmp /tmp/n_ref.npz /tmp/n_b.npz || exit 3
for rep in 1 2; do
  for v in prod nthS nthC nthB; do
    if [ $v = prod ]; then L=$N; else L=$PWD/abl/libfoto_$v.so; fi
    FOTO_LIB=$L FOTO_LIB_LAX=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-gn --no-stencil --steps 100 > $O/ab_nth_${v}_$rep.json 2> $O/ab_nth_${v}_$rep.err || { tail -5 $O/ab_nth_${v}_$rep.err; exit 4; }
    echo -n "$v r$rep "; python tools/show_bench.py $O/ab_nth_${v}_$rep.json
  done
done
rm -rf $O/prof_nthB
FOTO_LIB=$PWD/abl/libfoto_nthB.so FOTO_LIB_LAX=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_nthB -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stencil --no-gn --no-kernel-timing > $O/prof_nthB.log 2>&1 || exit 5
python3 - $O/prof_nthB/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "dct_fft" in r["Name"]: print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
