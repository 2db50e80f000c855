#!/bin/bash
# round-5: the w_t overlap -- mock-RCCL bit identity (incl. bench grid / C4 at W=8), then the
# compute proxy + communication model on the bench grid and C4
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_rccl_mock.py tests/test_gpu_parity.py -k "rccl or shard or virtual" -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/wt_tests.log 2>&1 || { tail -30 $O/wt_tests.log; exit 1; }
tail -2 $O/wt_tests.log
timeout -k 10 200 python -u tools/proxy_scaling.py --out $O/wt_proxy_bench.txt > $O/wt_proxy_bench.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/proxy_scaling.py --grid c4 --worlds 1,2,4,8 --steps 5 --warmup 2 --out $O/wt_proxy_c4.txt > $O/wt_proxy_c4.log 2>&1 || exit 3
grep -v '^\[' $O/wt_proxy_bench.txt; grep -v '^\[' $O/wt_proxy_c4.txt
