#!/bin/bash
# A round's GPU check: the whole -m gpu suite (prints kept), smoke, one default bench line
# without the CPU baselines.  tools/gpu_round.sh TAG   (from the repo root on the GPU box)
set -o pipefail
O=gpurun_out; tag="${1:-r06}"; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests_$tag.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 $O/tests_$tag.log; grep -E "^FAILED|^ERROR" $O/tests_$tag.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$tag.log 2>&1 || exit 3
tail -1 $O/smoke_$tag.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-gn --no-stencil > $O/bench_$tag.json 2> $O/bench_$tag.err || exit 4
python tools/show_bench.py $O/bench_$tag.json 2>/dev/null || tail -c 600 $O/bench_$tag.json
exit $rc
