#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_asr.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/x3t.log 2>&1; tail -2 gpurun_out/x3t.log; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/x3t.log | head -8
