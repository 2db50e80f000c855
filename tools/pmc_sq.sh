#!/bin/bash
# SQ counters (two passes of <= 8 SQ counters) for the bench's big kernels: instruction mix per wave,
# VALU / LDS busy, wave cycles (tools/pmc_sq_summary.py prints the table).  tools/pmc_sq.sh [KERNEL-REGEX]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
args="--steps 3 --warmup 1 --no-cpu-baseline --no-stencil --no-gn --no-kernel-timing"
re="${1:-k_gq_xhat|k_dct_fft|k_prox_rhs|k_gq_hist|k_dct_t_|k_gq_cg}"
rm -rf $O/pmc_sq1 $O/pmc_sq2
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$re" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -f csv -d $O/pmc_sq1 -o run -- python3 bench.py $args > $O/pmc_sq1.log 2>&1 || { tail -5 $O/pmc_sq1.log; exit 2; }
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$re" --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F64 -f csv -d $O/pmc_sq2 -o run -- python3 bench.py $args > $O/pmc_sq2.log 2>&1 || { tail -5 $O/pmc_sq2.log; exit 3; }
python3 tools/pmc_sq_summary.py $O/pmc_sq1 $O/pmc_sq2
