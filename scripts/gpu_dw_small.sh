#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 150 python3 scripts/dw_small_bench.py > gpurun_out/dw_small2.log 2>&1 || { tail -5 gpurun_out/dw_small2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/dw_small2.log
