#!/bin/bash
# Round evidence: GPU tests, the default bench line, kernel trace + stats,
# FETCH_SIZE / WRITE_SIZE passes, per-form summaries (durations, traffic), the
# headline step's timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gputest.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
tail -2 gpurun_out/gputest.log
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1 || exit $?
echo "bench ok"
# SKIP_PMC=1: kernel trace only (the committed profiles/pmc_summary.json stays)
SKIP_PMC=${SKIP_PMC:-0} bash scripts/prof_round.sh || exit 1
TR=$(ls gpurun_out/prof/*kernel_trace.csv gpurun_out/prof/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/trace_summary.py "$TR" gpurun_out/trace_summary.json > /dev/null || exit 1
if [ "${SKIP_PMC:-0}" != 1 ]; then
  python3 scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_summary.json > /dev/null || exit 1
fi
bash scripts/gpu_trace.sh || exit 1
python3 scripts/step_timeline.py $(ls gpurun_out/tr8192/*kernel_trace.csv gpurun_out/tr8192/*/*kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/step8192_timeline.txt || exit 1
echo "profile ok"
