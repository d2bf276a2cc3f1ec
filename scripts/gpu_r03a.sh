#!/bin/bash
# Round-3 first evidence run: GPU tests, then the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gputest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_full.log; exit 1; }
tail -c 6000 gpurun_out/bench_full.log
timeout -k 10 120 ./scripts/bin/wstream > gpurun_out/wstream.log 2>&1 || exit $?
cat gpurun_out/wstream.log
