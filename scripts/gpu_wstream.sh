#!/bin/bash
# weight-stream ceiling microbenchmark + L2 hit rate of the lockstep fused kernel
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 ./scripts/bin/wstream > gpurun_out/wstream.log 2>&1 || exit $?

timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_l2 -o l2 --output-format csv -- python3 scripts/vs_once.py 65536 3 > gpurun_out/pmc_l2.log 2>&1 || exit $?
export MOG_VS_PHASES=2
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_l2d -o l2d --output-format csv -- python3 scripts/vs_once.py 65536 3 > gpurun_out/pmc_l2d.log 2>&1
