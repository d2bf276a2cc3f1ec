#!/bin/bash
# early decoder weight gradients (MOG_WGRAD_EARLY) A/B on the fp32 step, tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for e in 1 0 1 0; do
  MOG_WGRAD_EARLY=$e timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 --extras 0 --roofline-batch 0 > gpurun_out/r04m_$e.log 2>&1 || { tail -3 gpurun_out/r04m_$e.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r04m_$e.log').read().strip().splitlines()[-1]);print('early $e: fp32 step', round(d['ms_per_step'],3), 'ms')"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_graph.py tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04m_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r04m_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/r04m_tests.log | head
[ $rc -le 1 ] || exit $rc
rm -rf gpurun_out/tr8192
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr8192 -o run -- python3 bench.py --steps 6 --warmup 2 --cpu-baseline 0 --extras 0 --roofline-batch 0 --batch 8192 > gpurun_out/tr8192.log 2>&1 || { tail -3 gpurun_out/tr8192.log; exit 1; }
f=$(ls gpurun_out/tr8192/*kernel_trace.csv gpurun_out/tr8192/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/step_timeline.py "$f" > gpurun_out/step8192_timeline.txt && python3 scripts/prof_step.py "$f" > gpurun_out/step8192.txt && tail -1 gpurun_out/step8192.txt
