#!/bin/bash
# fused-step per-phase timing (output-layer passes split) + headline step traces
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -u scripts/vs_phases.py 65536 timing > gpurun_out/vsdiag_t31.log 2>&1 || exit $?
cat gpurun_out/vsdiag_t31.log
bash scripts/gpu_trace.sh || exit 1
cat gpurun_out/step8192.txt gpurun_out/step64.txt
