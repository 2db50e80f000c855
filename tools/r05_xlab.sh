#!/bin/bash
# (the FOTO_GQ_XLAB lab switch was removed from foto_gauss.inc after this measurement; results in profiles/r05_xhat_mono_ab.txt)
# (lab) k_gq_xhat without its Clenshaw (1) or without bins and Clenshaw (2): what the kernel's loads
# and stores cost alone -- kernel trace of the default bench with each lab build (results wrong)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
for v in prod xlab1 xlab2; do
  if [ $v = prod ]; then L=$PWD/optical-flow-optimal-transport_amd/foto/libfoto.so; else L=$PWD/abl/libfoto_$v.so; fi
  rm -rf $O/prof_$v
  FOTO_LIB=$L FOTO_LIB_LAX=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_$v -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stencil --no-gn --no-kernel-timing > $O/prof_$v.log 2>&1 || exit 5
  python3 - $O/prof_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_gq_xhat" in r["Name"] or "k_dct_t_inv_xhat" in r["Name"]: print(sys.argv[2], r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
done
