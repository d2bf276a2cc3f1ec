#!/bin/bash
# GPU tests (one process) then the default bench line; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ${TESTS:-} > gpurun_out/gputest.log 2>&1 || { tail -30 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
[ "${BENCH:-1}" = 1 ] || exit 0
timeout -k 10 500 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -c 3000 gpurun_out/bench.log
