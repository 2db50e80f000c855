#!/bin/bash
# k_prox_rhs chunk length (FOTO_PR_TCH) A/B on the default bench: 16 (default) vs 11 and 12
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/r05_ab.sh tch11 "FOTO_PR_TCH=16" "FOTO_PR_TCH=11" 2 || exit 3
bash tools/r05_ab.sh tch12 "FOTO_PR_TCH=16" "FOTO_PR_TCH=12" 2 || exit 4
