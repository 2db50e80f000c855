#!/bin/bash
# the sharded paths after a change to the slab <-> box all-to-all: virtual ranks, in-process RCCL,
# sharded Gauss, C4; then the compute-only proxy curves (bench grid and C4)
set -o pipefail
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -k "virtual or sharded or rccl or c4 or gauss or vr" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/a2a_tests.log 2>&1 || { tail -30 $O/a2a_tests.log; exit 1; }
tail -1 $O/a2a_tests.log
timeout -k 10 240 python tools/proxy_scaling.py --out $O/r04i_proxy_scaling.txt > /dev/null 2>&1 || exit 1
head -9 $O/r04i_proxy_scaling.txt
timeout -k 10 300 python tools/proxy_scaling.py --grid c4 --steps 5 --warmup 2 --out $O/r04i_proxy_scaling_c4.txt > /dev/null 2>&1 || exit 1
head -9 $O/r04i_proxy_scaling_c4.txt
