#!/bin/bash
# (experiment) the inverse y / x DCTs in plane groups on two streams (FOTO_INV_SPLIT): bit identity
# at the bench grid, then a same-box A/B on the default bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python - <<'PY' || exit 2
import os, sys, numpy as np
sys.path.insert(0, "optical-flow-optimal-transport_amd")
from foto.bb import BBSolver
from foto.synthetic import translating_gaussian
Nt, Nx, Ny = 32, 640, 480
rho0, rhoT = translating_gaussian(Nx, Ny)
out = {}
for v in ("0", "2", "4"):
    os.environ["FOTO_INV_SPLIT"] = v
    with BBSolver(rho0, rhoT, Nt, Nx, Ny, r=1.0, reg_epsilon=1e-2, cg_mode=3) as s:
        s.iterate(4, 0.0, stop_rules=False)
        out[v] = (np.array(s.cg_its), np.array(s.crit), s.phi())
for v in ("2", "4"):
    same = all(np.array_equal(a, b) for a, b in zip(out["0"], out[v]))
    print("split", v, "bit-identical", same)
    assert same
PY
bash tools/r05_ab.sh split "FOTO_INV_SPLIT=0" "FOTO_INV_SPLIT=2" 3 || exit 3
bash tools/r05_ab.sh split4 "FOTO_INV_SPLIT=0" "FOTO_INV_SPLIT=4" 2 || exit 4
