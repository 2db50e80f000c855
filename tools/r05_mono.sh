#!/bin/bash
# solution table in monomial form + Horner (FOTO_GQ_MONO=19, default) against Chebyshev + Clenshaw
# (FOTO_GQ_MONO=0 build): difference of phi / crit / CG counts at the bench grid, the Gauss and
# parity GPU tests, same-box A/B, x^ kernel time
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
N=$PWD/optical-flow-optimal-transport_amd/foto/libfoto.so; C=$PWD/abl/libfoto_mono0.so
FOTO_LIB=$N timeout -k 10 120 python tools/bitcmp.py save /tmp/m_new.npz 32 640 480 10 || exit 2
FOTO_LIB=$C FOTO_LIB_LAX=1 timeout -k 10 120 python tools/bitcmp.py save /tmp/m_old.npz 32 640 480 10 || exit 2
python - <<'PY'
import numpy as np
a, b = np.load("/tmp/m_new.npz"), np.load("/tmp/m_old.npz")
print("cg equal:", np.array_equal(a["cg"], b["cg"]), "crit max rel:", float(np.max(np.abs(a["crit"] - b["crit"]) / np.abs(b["crit"]))),
      "phi max abs / max|phi|:", float(np.max(np.abs(a["phi"] - b["phi"])) / np.max(np.abs(b["phi"]))))
PY
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gauss.py tests/test_gpu_parity.py tests/test_gpu_configs.py > $O/m_tests.log 2>&1 || { tail -30 $O/m_tests.log; exit 4; }
tail -1 $O/m_tests.log
for rep in 1 2 3; do
  for v in new old; do
    if [ $v = new ]; then L=$N; else L=$C; fi
    FOTO_LIB=$L FOTO_LIB_LAX=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-gn --no-stencil --steps 100 > $O/ab_mono_${v}_$rep.json 2> $O/ab_mono_${v}_$rep.err || { tail -5 $O/ab_mono_${v}_$rep.err; exit 5; }
    echo -n "$v r$rep "; python tools/show_bench.py $O/ab_mono_${v}_$rep.json
  done
done
rm -rf $O/prof_mono
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_mono -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stencil --no-gn --no-kernel-timing > $O/prof_mono.log 2>&1 || exit 6
python3 - $O/prof_mono/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_gq_xhat" in r["Name"] or "k_gq_qtab" in r["Name"]: print(r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
