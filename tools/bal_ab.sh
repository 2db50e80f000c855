#!/bin/bash
# balanced prox work split: parity tests under FOTO_PR_BAL, then a same-box A/B against the
# previous build (FOTO_LIB) and the legacy split of this build
set -o pipefail
O=gpurun_out
FOTO_PR_BAL=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipe.py tests/test_gpu_rccl_mock.py -q -x -k "prox or pipe_stop or bit_identical or c4" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/bal_tests.log 2>&1 || { tail -30 $O/bal_tests.log; exit 1; }
tail -1 $O/bal_tests.log
for rep in 1 2; do
  for setting in "FOTO_LIB=$PWD/build_ab/libfoto_head.so FOTO_LIB_LAX=1" "FOTO_PR_BAL=0" "FOTO_PR_BAL=1" "FOTO_PR_BAL=2"; do
    env $setting timeout -k 10 120 python bench.py --no-cpu-baseline --no-stencil --no-gn --steps 40 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']
print('${setting##*/}', d['value'], d['ms_per_step'], {n: round(v['avg_us'],1) for n,v in k.items()})" || exit 1
  done
done
