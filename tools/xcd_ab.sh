#!/bin/bash
# A/B of the histogram's XCD-grouped chunk order (FOTO_GQ_XCD): tests, bench, and per setting a
# kernel-trace pass and a FETCH_SIZE pass (CSV under gpurun_out/xcd_*).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gauss.py tests/test_gpu_pipe.py tests/test_gpu_rccl_mock.py -q -x -k "not c4_w8" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/xcd_tests.log 2>&1 || { tail -30 $O/xcd_tests.log; exit 1; }
tail -1 $O/xcd_tests.log
timeout -k 10 300 bash tools/ab_env.sh FOTO_GQ_XCD=1 FOTO_GQ_XCD=0 > $O/xcd_ab.txt 2>&1 || { cat $O/xcd_ab.txt; exit 1; }
cat $O/xcd_ab.txt
args="--steps 10 --warmup 2 --no-cpu-baseline --no-stencil --no-gn --no-kernel-timing"
for v in 1 0; do
  rm -rf $O/xcd_kt$v $O/xcd_f$v
  FOTO_GQ_XCD=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/xcd_kt$v -o run -- python3 bench.py $args > $O/xcd_kt$v.log 2>&1 || exit 1
  FOTO_GQ_XCD=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/xcd_f$v -o run -- python3 bench.py $args > $O/xcd_f$v.log 2>&1 || exit 1
done
echo done
