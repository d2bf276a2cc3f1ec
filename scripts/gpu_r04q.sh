#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_graph.py tests/test_gpu_torch_ops.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04q_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r04q_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/r04q_tests.log | head
[ $rc -le 1 ] || exit $rc
for i in 1 2; do timeout -k 10 120 python3 scripts/b64_graph_trace.py 64 2>&1 | grep ms/step; done
