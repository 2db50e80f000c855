#!/bin/bash
# interleaved same-box A/B of the in-tree build against variant libraries (prox parity first)
# usage: tools/ab3.sh NAME=path.so [NAME=path.so ...]
set -o pipefail
O=gpurun_out
for v in "$@"; do
  n=${v%%=*}; lib=${v#*=}
  FOTO_LIB=$PWD/$lib FOTO_LIB_LAX=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gauss.py tests/test_gpu_pipe.py -q -x -k "${ABK:-prox or stepb}" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/ab3_tests_$n.log 2>&1 || { tail -20 $O/ab3_tests_$n.log; exit 1; }
  echo "$n: $(tail -1 $O/ab3_tests_$n.log)"
done
bash tools/ab_lib.sh base=optical-flow-optimal-transport_amd/foto/libfoto.so "$@" -- python bench.py --no-cpu-baseline --no-gn --no-stencil --steps 40 > $O/ab3.txt 2>&1 || exit 1
python - $O/ab3.txt <<'PY'
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
