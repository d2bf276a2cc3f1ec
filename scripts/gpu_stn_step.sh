#!/bin/bash
# STN backward at the train-step rows (stand-alone, per-wave phases) and one
# fp32 train step's kernel timeline at B = 8192
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/bench_stn.py 24576 > gpurun_out/stn24576.log 2>&1 || { tail -5 gpurun_out/stn24576.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stn24576.log
rm -rf gpurun_out/tr8192
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr8192 -o run -- python3 bench.py --steps 6 --warmup 2 --cpu-baseline 0 --extras 0 --roofline-batch 0 --batch 8192 > gpurun_out/tr8192.log 2>&1 || { tail -3 gpurun_out/tr8192.log; exit 1; }
f=$(ls gpurun_out/tr8192/*kernel_trace.csv gpurun_out/tr8192/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/step_timeline.py "$f" > gpurun_out/step8192_timeline.txt && python3 scripts/prof_step.py "$f" > gpurun_out/step8192.txt && tail -40 gpurun_out/step8192.txt
