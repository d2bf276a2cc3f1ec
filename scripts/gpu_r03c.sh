#!/bin/bash
# fp32 fused-step phases + the batch-64 step after the small-batch switch
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 200 python -u scripts/f32_time.py 24576 > gpurun_out/f32_time.log 2>&1 || exit $?
cat gpurun_out/f32_time.log
timeout -k 10 200 python -u bench.py --batch 64 --steps 50 --warmup 5 --extras 0 --cpu-baseline 0 --roofline-batch 0 > gpurun_out/b64.log 2>&1 || exit $?
tail -1 gpurun_out/b64.log | cut -c1-400
