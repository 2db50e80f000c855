#!/bin/bash
# Interleaved same-box A/B of library builds (FOTO_LIB): tools/ab_lib.sh "name=path.so" ... -- cmd
# Each library runs the command twice, interleaved with the others.
libs=(); while [ "$1" != "--" ] && [ -n "$1" ]; do libs+=("$1"); shift; done; shift
for rep in 1 2; do
  for v in "${libs[@]}"; do
    n=${v%%=*}; lib=${v#*=}
    echo "== $n (rep $rep)"
    FOTO_LIB=$PWD/$lib FOTO_LIB_LAX=1 timeout -k 10 300 "$@" || exit $?
  done
done
