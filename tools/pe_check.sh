set -o pipefail
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_batch.py tests/test_gpu_rccl_mock.py tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pe_tests.log 2>&1 || { tail -30 $O/pe_tests.log; exit 1; }
tail -1 $O/pe_tests.log
bash tools/ab_env40.sh FOTO_PHASE_EV=1 FOTO_POLL=0 FOTO_DUMMY=0 || exit 1
timeout -k 10 200 python bench.py --no-stencil --no-gn --no-cpu-baseline --steps 20 > $O/pe_bench.json || exit 1
python tools/show_bench.py $O/pe_bench.json; python -c "import json;d=json.loads(open('$O/pe_bench.json').read().strip().splitlines()[-1]);print(d['phase_ms'])"
