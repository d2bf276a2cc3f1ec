#!/bin/bash
# Round-4 evidence: full GPU suite, the default bench line, then the profile
# (kernel trace of the bench, per-workload trace + FETCH / WRITE passes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gputest.log 2>&1; rc=$?
tail -3 gpurun_out/r04_gputest.log
[ $rc -le 1 ] || exit $rc; grep -E "^(FAILED|ERROR)" gpurun_out/r04_gputest.log | head -20
timeout -k 10 500 python bench.py > gpurun_out/r04_bench.log 2>&1 || { tail -5 gpurun_out/r04_bench.log; exit 1; }
echo "bench ok"
bash scripts/prof_r04.sh
