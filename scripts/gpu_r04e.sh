#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "stale or captured_workspace" > gpurun_out/r04e_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04e_tests.log
[ $rc -le 1 ] || exit $rc; grep -E "^(FAILED|E  )" gpurun_out/r04e_tests.log | head -10
timeout -k 10 300 python -u scripts/x3_lib_bench.py 2>&1 | grep -v amdgpu.ids
