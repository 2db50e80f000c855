#!/bin/bash
# quick same-box A/B of one variant library against the in-tree build: the variant's stepB/prox
# parity tests, then interleaved bench runs.  usage: tools/ab_quick.sh NAME=path.so [pytest -k expr]
set -o pipefail
O=gpurun_out
v="$1"; n=${v%%=*}; lib=${v#*=}; kx="${2:-stepb or prox}"
FOTO_LIB=$PWD/$lib FOTO_LIB_LAX=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipe.py -q -x -k "$kx" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/abq_tests_$n.log 2>&1 || { tail -30 $O/abq_tests_$n.log; exit 1; }
tail -1 $O/abq_tests_$n.log
bash tools/ab_lib.sh base=optical-flow-optimal-transport_amd/foto/libfoto.so "$v" -- python bench.py --no-cpu-baseline --no-gn --no-stencil --steps 40 > $O/abq_$n.txt 2>&1 || exit 1
python - $O/abq_$n.txt <<'PY'
import json, sys
name = None
for ln in open(sys.argv[1]):
    if ln.startswith("=="):
        name = ln.strip()
    elif ln.startswith("{"):
        d = json.loads(ln)
        k = {a: round(b["avg_us"], 1) for a, b in d.get("kernels", {}).items()}
        print(name, d["value"], d["ms_per_step"], k)
PY
