#!/bin/bash
# kernel-trace profile of a short default bench under an env setting; top kernels printed
#   tools/r05_prof.sh TAG ["ENV=VAL ..."]
set -o pipefail
tag=$1; envs=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf gpurun_out/prof_$tag
env $envs timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --steps 10 \
    --warmup 2 --no-cpu-baseline --no-stencil --no-gn --no-kernel-timing > gpurun_out/prof_$tag.log 2>&1 || { tail -5 gpurun_out/prof_$tag.log; exit 5; }
f=$(find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:18]:
    print(f"{r['Name'][:80]:80s} n={r['Calls']:>5} avg={float(r['AverageNs']) / 1e3:9.2f}us")
PY
