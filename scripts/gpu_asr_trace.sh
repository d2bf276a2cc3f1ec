#!/bin/bash
# kernel sums of the fp32 ASR train step at B = 8192 (prof_step's per-kernel table)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
rm -rf gpurun_out/trasr
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trasr -o run -- python3 scripts/asr_steps.py > gpurun_out/trasr.log 2>&1 || { tail -3 gpurun_out/trasr.log; exit 1; }
f=$(ls gpurun_out/trasr/*kernel_trace.csv gpurun_out/trasr/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/prof_step.py "$f" > gpurun_out/asr_step.txt && head -30 gpurun_out/asr_step.txt && tail -1 gpurun_out/asr_step.txt
python3 scripts/step_timeline.py "$f" > gpurun_out/asr_timeline.txt
