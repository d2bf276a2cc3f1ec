#!/bin/bash
# x-rows gradient kernel variants (scripts/x1_sweep.py), one process each,
# each under its own time limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for V in ${VARS:--1 0 1 2 3}; do
  MOG_X3P_VAR=$V timeout -k 10 120 python3 -u scripts/x1_sweep.py >> gpurun_out/x1_sweep.log 2>&1 || { echo "variant $V failed"; tail -20 gpurun_out/x1_sweep.log; exit 1; }
done
cat gpurun_out/x1_sweep.log
