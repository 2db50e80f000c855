#!/bin/bash
# One profiling pass of the bench workload, as MI355X_MICROARCH.md's HBM section prescribes:
# kernel trace + stats in one run, FETCH_SIZE and WRITE_SIZE each in a run of their own, the
# calibration streams (tools/calib_fetch) under the same two counters, then the summary.
# usage: tools/profile_round.sh TAG [bench args...]      (run from the repo root on the GPU box)
set -o pipefail
tag="$1"; shift
args="${*:---steps 10 --warmup 2 --no-cpu-baseline --no-stencil}"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
rm -rf $O/prof_kt $O/prof_fetch $O/prof_write $O/cal_fetch $O/cal_write
timeout -k 10 240 python3 bench.py $args > $O/bench_full.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_kt -o run -- python3 bench.py $args --no-kernel-timing > $O/prof_kt.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/prof_fetch -o run -- python3 bench.py $args --no-kernel-timing > $O/prof_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/prof_write -o run -- python3 bench.py $args --no-kernel-timing > $O/prof_write.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/cal_fetch -o run -- tools/calib_fetch > $O/cal_fetch.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/cal_write -o run -- tools/calib_fetch > $O/cal_write.log 2>&1 || exit $?
# the bench command itself (timed loop + kernel-timing pass) under the kernel trace: the dominant
# kernel's launches of each segment (tools/prox_segments.py)
rm -rf $O/prof_kt2
timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d $O/prof_kt2 -o run -- python3 bench.py $args > $O/prof_kt2.log 2>&1 || exit $?
python3 tools/prox_segments.py $O/prof_kt2/run_kernel_trace.csv 10 2 $O/prox_loop_trace.json \
    "profiles/${tag}_prox_segments.txt (rocprofv3 --kernel-trace of bench.py $args: k_prox_rhs in the timed loop vs in the HIP-event timing pass, same run)" \
    > $O/prox_segments.txt || exit $?
python3 tools/summarize_profile.py --tag "$tag" --kt $O/prof_kt --fetch $O/prof_fetch --write $O/prof_write \
    --calib-fetch $O/cal_fetch --calib-write $O/cal_write --bench $O/bench_full.log --out $O/profiles_new
