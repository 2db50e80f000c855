#!/bin/bash
# histogram variants: kernel-trace stats per (library, FOTO_GQ_TABL) -> gq_hist average
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
args="--steps 10 --warmup 2 --no-cpu-baseline --no-stencil --no-gn --no-kernel-timing"
FOTO_LIB=$PWD/build_ab/libfoto_pe8.so FOTO_LIB_LAX=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_gauss.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/hab_tests.log 2>&1 || { tail -20 $O/hab_tests.log; exit 1; }
tail -1 $O/hab_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_gauss.py tests/test_gpu_pipe.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/hab_tests2.log 2>&1 || { tail -20 $O/hab_tests2.log; exit 1; }
tail -1 $O/hab_tests2.log
for rep in 1 2; do
for lib in base=optical-flow-optimal-transport_amd/foto/libfoto.so pe8=build_ab/libfoto_pe8.so pe4=build_ab/libfoto_pe4.so; do
  n=${lib%%=*}; l=${lib#*=}
  for t in 1 0; do
    d=$O/hab_${n}_t${t}_$rep; rm -rf $d
    FOTO_GQ_TABL=$t FOTO_LIB=$PWD/$l FOTO_LIB_LAX=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $d -o run -- python3 bench.py $args > $d.log 2>&1 || exit 1
    python3 - $d/run_kernel_stats.csv "$n tabl=$t rep=$rep" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_gq_hist_perm' in r['Name']:
        print(sys.argv[2], 'gq_hist', round(float(r['AverageNs']) / 1e3, 2), 'us')
PY
  done
done
done
