#!/bin/bash
# Round profile of the bench command: kernel trace + stats, then one PMC pass
# per counter (FETCH_SIZE and WRITE_SIZE can not share a pass), each under
# its own time limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD="python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 --roofline-launches 5"
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- $CMD > gpurun_out/prof.log 2>&1 || { echo "trace failed"; exit 1; }
echo "trace ok"
[ "${SKIP_PMC:-0}" = 1 ] && exit 0
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- $CMD > gpurun_out/pmcf.log 2>&1 || { echo "fetch pass failed"; exit 1; }
echo "fetch ok"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- $CMD > gpurun_out/pmcw.log 2>&1 || { echo "write pass failed"; exit 1; }
echo "write ok"
