#!/bin/bash
# Round-4 GPU session: diagnosis, the GPU tests (all of them, failures listed), the compute-only
# proxy curves at the bench grid and C4, then the profile pass (kernel trace + PMC).
# usage (from the repo root on the GPU box): tools/r04_gpu.sh TAG
set -o pipefail
tag="${1:-r04}"
O=gpurun_out
mkdir -p $O
timeout -k 10 120 python tools/dbg_redo.py > $O/dbg_redo.txt 2>&1; echo "dbg rc=$?"; cat $O/dbg_redo.txt
[ -x tools/gqnodes_lab ] && { (cd tools && timeout -k 10 60 ./gqnodes_lab 50 3 && timeout -k 10 60 ./gqnodes_lab 50 1) > $O/gqnodes_lab.txt 2>&1; cat $O/gqnodes_lab.txt; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests_$tag.log 2>&1
echo "tests rc=$?"; tail -4 $O/tests_$tag.log; grep -E "^FAILED|eps 1e-3|C2 mode|C4 gauss|C1 mode" $O/tests_$tag.log
if [ -n "$AB" ]; then   # AB="name=path.so ...": interleaved same-box A/B of library builds
  bash tools/ab_lib.sh base=optical-flow-optimal-transport_amd/foto/libfoto.so $AB -- python bench.py --no-cpu-baseline --no-gn --no-stencil --steps 40 > $O/ab_$tag.txt 2>&1
  echo "ab rc=$?"; python - $O/ab_$tag.txt <<'PY'
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
fi
[ -n "$SKIP_PROXY" ] || {
timeout -k 10 240 python tools/proxy_scaling.py --out $O/${tag}_proxy_scaling.txt > /dev/null 2>&1; echo "proxy rc=$?"; head -12 $O/${tag}_proxy_scaling.txt
timeout -k 10 300 python tools/proxy_scaling.py --grid c4 --steps 5 --warmup 2 --out $O/${tag}_proxy_scaling_c4.txt > /dev/null 2>&1; echo "proxy c4 rc=$?"; head -12 $O/${tag}_proxy_scaling_c4.txt
}
[ -n "$SKIP_PROF" ] || { bash tools/profile_round.sh $tag > $O/prof_$tag.txt 2>&1; echo "prof rc=$?"; tail -5 $O/prof_$tag.txt; }
exit 0
