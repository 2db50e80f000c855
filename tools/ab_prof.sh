#!/bin/bash
# Kernel-trace the bench under several library builds (FOTO_LIB): tools/ab_prof.sh name=path.so ...
# Writes gpurun_out/abp_<name>/ (rocprofv3 kernel stats); run from the repo root on the GPU box.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in "$@"; do
    n=${v%%=*}; lib=${v#*=}
    rm -rf gpurun_out/abp_$n
    FOTO_LIB=$PWD/$lib FOTO_LIB_LAX=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/abp_$n -o run \
        -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stencil --no-gn --no-kernel-timing \
        > gpurun_out/abp_$n.log 2>&1 || exit $?
done
