#!/bin/bash
# GPU tests (one process; TESTS narrows them) then the batch-64 graph trace
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/quick_tests.log 2>&1
rc=$?
tail -4 gpurun_out/quick_tests.log
[ $rc = 0 ] || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/quick_tests.log | head; exit $rc; }
[ "${B64:-1}" = 1 ] && bash scripts/gpu_b64.sh | tail -3
exit 0
