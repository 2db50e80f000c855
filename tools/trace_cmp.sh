#!/bin/bash
# Kernel traces of the bench workload under two settings of an env knob (A/B), written to
# gpurun_out/trace_<name>/.  usage: tools/trace_cmp.sh NAME "ENV=VAL ..." [bench args]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
name="$1"; envs="$2"; shift 2
args="${*:---steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing}"
rm -rf gpurun_out/trace_$name
env $envs true   # validate
export $envs
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/trace_$name -o run -- python3 bench.py $args > gpurun_out/trace_$name.log 2>&1
