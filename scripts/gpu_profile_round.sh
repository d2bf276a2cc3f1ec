#!/bin/bash
# Round evidence: GPU tests, the default bench line, kernel trace + stats,
# FETCH_SIZE / WRITE_SIZE passes, SQ passes of the STN backward.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gputest.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1 || exit $?
bash scripts/prof_round.sh || exit 1
bash scripts/pmc_stn_sq.sh 24576 || exit 1
