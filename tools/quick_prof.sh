#!/bin/bash
# Quick GPU iteration: the Gauss CG tests, a short bench and a kernel-trace profile of it.
# usage (on the GPU box, from the repo root): tools/quick_prof.sh [extra pytest files...]
set -o pipefail
tests="${*:-tests/test_gpu_gauss.py}"
tools/gpu_steps.sh "300|qtests|python -u -m pytest $tests -x -q --timeout 200 --timeout-method thread" \
    "200|bench3|python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gn --no-stencil" || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf gpurun_out/prof_g3
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_g3 -o run -- python3 bench.py --steps 10 \
    --warmup 2 --no-cpu-baseline --no-stencil --no-gn --no-kernel-timing > gpurun_out/prof_g3.log 2>&1
