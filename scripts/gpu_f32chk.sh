#!/bin/bash
# fp32 fused step: parity tests + phase timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_f32.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/f32chk.log 2>&1 || { tail -30 gpurun_out/f32chk.log; exit 1; }
tail -1 gpurun_out/f32chk.log
timeout -k 10 200 python -u scripts/f32_time.py 24576 > gpurun_out/f32_time.log 2>&1 || exit $?
cat gpurun_out/f32_time.log
