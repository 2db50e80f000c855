#!/bin/bash
# round 5: product tests, then the 64x16 two-voxel k_prox_rhs build (abl/libfoto_pr16.so) against
# the product: its parity tests, then interleaved benches (prox event time in each line)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gauss.py \
    tests/test_gpu_pipe.py tests/test_gpu_parity.py > $O/r05p_tests.log 2>&1 || { tail -30 $O/r05p_tests.log; exit 3; }
tail -2 $O/r05p_tests.log
FOTO_LIB=$PWD/abl/libfoto_pr16.so FOTO_LIB_LAX=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipe.py > $O/r05p_tests_pr16.log 2>&1 || { tail -30 $O/r05p_tests_pr16.log; exit 4; }
tail -2 $O/r05p_tests_pr16.log
for rep in 1 2; do
  for v in main=optical-flow-optimal-transport_amd/foto/libfoto.so pr16=abl/libfoto_pr16.so; do
    n=${v%%=*}; lib=${v#*=}
    FOTO_LIB=$PWD/$lib FOTO_LIB_LAX=1 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/r05p_bench_${n}_$rep.json 2> $O/r05p_bench_${n}_$rep.err || exit 5
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline',{}); print(sys.argv[2], round(d['value'],1), 'it/s; prox us', r.get('avg_launch_us'), 'frac', r.get('frac'))" $O/r05p_bench_${n}_$rep.json $n
  done
done
