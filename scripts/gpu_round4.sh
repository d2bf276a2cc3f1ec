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
# the headline step's kernel timeline (one fp32 step of a profiled bench run)
rm -rf gpurun_out/tr8192
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr8192 -o run -- python3 bench.py --steps 6 --warmup 2 --cpu-baseline 0 --extras 0 --roofline-batch 0 --batch 8192 > gpurun_out/tr8192.log 2>&1 || { tail -3 gpurun_out/tr8192.log; exit 1; }
f=$(ls gpurun_out/tr8192/*kernel_trace.csv gpurun_out/tr8192/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/step_timeline.py "$f" > gpurun_out/step8192_timeline.txt && python3 scripts/prof_step.py "$f" > gpurun_out/step8192.txt && tail -1 gpurun_out/step8192.txt
