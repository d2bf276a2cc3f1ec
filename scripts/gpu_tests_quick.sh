#!/bin/bash
# the GPU suites the stream / prologue changes touch
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_x3.py tests/test_gpu_parity.py tests/test_gpu_dp.py tests/test_gpu_asr.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/quick_tests.log 2>&1; rc=$?
tail -3 gpurun_out/quick_tests.log; exit $rc
