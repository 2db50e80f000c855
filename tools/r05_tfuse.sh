#!/bin/bash
# fused x^ + inverse t-DCT (FOTO_GQ_TFUSE=1): bit-identity test, env A/B on the default bench, the
# 6-deep prefetch build, and a kernel trace of the fused default
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gauss.py -k tfuse \
    > gpurun_out/r05_tfuse_tests.log 2>&1 || { tail -30 gpurun_out/r05_tfuse_tests.log; exit 2; }
tail -1 gpurun_out/r05_tfuse_tests.log
bash tools/r05_ab.sh tfuse "FOTO_GQ_TFUSE=0" "FOTO_GQ_TFUSE=1" 2 || exit 3
for r in 1 2; do
  FOTO_LIB=$PWD/abl/libfoto_tf6.so FOTO_GQ_TFUSE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-gn --no-stencil --steps 100 > gpurun_out/ab_tf6_$r.json 2>/dev/null || exit 4
  echo -n "tf6 r$r "; python tools/show_bench.py gpurun_out/ab_tf6_$r.json
done
bash tools/r05_prof.sh tfuse "FOTO_GQ_TFUSE=1" || exit 5
