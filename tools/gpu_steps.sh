#!/bin/bash
# Run GPU steps in order, each under its own time limit.  A step that exits 0 or 1 (test
# failures) lets the next one run; a timeout, abort, segfault or kill ends the script.
# usage: tools/gpu_steps.sh "SECONDS|name|command" ...
mkdir -p gpurun_out
for spec in "$@"; do
    secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
    echo "=== [$name] $cmd (limit ${secs}s) $(date +%T)"
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "=== [$name] exit $rc $(date +%T)"
    tail -n 25 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "=== stopping: step $name ended with $rc"
        exit $rc
    fi
done
