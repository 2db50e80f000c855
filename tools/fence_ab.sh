#!/bin/bash
# fence-free timing / sync events: GPU tests of the loop, then a same-box A/B
set -o pipefail
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_batch.py tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/fence_tests.log 2>&1 || { tail -30 $O/fence_tests.log; exit 1; }
tail -1 $O/fence_tests.log
bash tools/ab_env40.sh FOTO_KT_FENCE=1 FOTO_SYNC_FENCE=1 FOTO_DUMMY=0 FOTO_PHASE_EV=1
