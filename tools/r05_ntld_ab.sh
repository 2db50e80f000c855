#!/bin/bash
# k_prox_rhs ring-voxel mu loads: non-temporal (product, FOTO_PR_NTLD=2) vs plain (abl/libfoto_ntld1.so):
# interleaved benches, then one FETCH_SIZE and one WRITE_SIZE pass of each (separate runs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
for rep in 1 2; do
  for v in nt2=optical-flow-optimal-transport_amd/foto/libfoto.so nt1=abl/libfoto_ntld1.so; do
    n=${v%%=*}; lib=${v#*=}
    FOTO_LIB=$PWD/$lib FOTO_LIB_LAX=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-gn --no-stencil > $O/r05n_bench_${n}_$rep.json 2> $O/r05n_bench_${n}_$rep.err || exit 5
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['value'],1), 'it/s; prox us', r.get('avg_launch_us'))" $O/r05n_bench_${n}_$rep.json $n
  done
done
for v in nt2=optical-flow-optimal-transport_amd/foto/libfoto.so nt1=abl/libfoto_ntld1.so; do
  n=${v%%=*}; lib=${v#*=}
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf $O/r05n_$n_$c
    FOTO_LIB=$PWD/$lib FOTO_LIB_LAX=1 timeout -s KILL 120 rocprofv3 --pmc $c -f csv -d $O/r05n_${n}_$c -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stencil --no-gn --no-kernel-timing > $O/r05n_${n}_$c.log 2>&1 || exit 6
  done
done
python3 - <<'PY'
import csv, glob, collections
for n in ("nt2", "nt1"):
    out = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(f"gpurun_out/r05n_{n}_{c}/**/*counter_collection.csv", recursive=True)[0]
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "k_prox_rhs" in r["Kernel_Name"]:
                acc[r.get("Dispatch_Id", r.get("Correlation_Id"))].append(float(r["Counter_Value"]))
        vals = [sum(v) for v in acc.values()]
        out[c] = sum(vals) / len(vals)
    # gfx950: FETCH_SIZE counts half the bytes of wide loads (calibrated 2.000 in tools/calib_fetch), WRITE_SIZE 1.000
    mb = (2.0 * out["FETCH_SIZE"] + out["WRITE_SIZE"]) * 1024 / 1e6
    print(f"{n}: k_prox_rhs FETCH_SIZE {out['FETCH_SIZE']:.0f} KiB, WRITE_SIZE {out['WRITE_SIZE']:.0f} KiB -> {mb:.1f} MB per launch (629.1 algorithmic)")
PY
