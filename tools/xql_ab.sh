#!/bin/bash
# x-hat table rows in LDS (FOTO_GQ_XQL): the Gauss / pipe / configs / parity GPU tests, then a same-box A/B
set -o pipefail
O=gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_gauss.py tests/test_gpu_pipe.py tests/test_gpu_configs.py tests/test_gpu_parity.py -q -x -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/xql_tests.log 2>&1 || { tail -30 $O/xql_tests.log; exit 1; }
tail -1 $O/xql_tests.log; grep -E "^eps|C1 mode 3" $O/xql_tests.log
bash tools/ab_env40.sh FOTO_GQ_XQL=0 FOTO_GQ_XQL=17
