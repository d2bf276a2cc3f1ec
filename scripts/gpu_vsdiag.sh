#!/bin/bash
# Fused bf16 step diagnostics: masked-phase launch times, per-phase in-kernel
# timing (all phases / dense only), L2 hit rates (all / dense only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VS_MASKS=31,2,3,10,11,0 timeout -k 10 200 python3 -u scripts/vs_phases.py 65536 > gpurun_out/vsdiag_masks.log 2>&1 || exit $?
timeout -k 10 200 python3 -u scripts/vs_phases.py 65536 timing > gpurun_out/vsdiag_t31.log 2>&1 || exit $?
MOG_VS_PHASES=2 timeout -k 10 200 python3 -u scripts/vs_phases.py 65536 timing > gpurun_out/vsdiag_t2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_l2 -o l2 --output-format csv -- python3 scripts/vs_once.py 65536 3 > gpurun_out/pmc_l2.log 2>&1 || exit $?
MOG_VS_PHASES=2 timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_l2d -o l2d --output-format csv -- python3 scripts/vs_once.py 65536 3 > gpurun_out/pmc_l2d.log 2>&1 || exit $?
cat gpurun_out/vsdiag_masks.log gpurun_out/vsdiag_t31.log gpurun_out/vsdiag_t2.log
