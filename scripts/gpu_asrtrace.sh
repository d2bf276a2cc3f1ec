#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
rm -rf gpurun_out/trasr
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trasr -o run -- python3 scripts/asr_trace.py 8192 fp32 > gpurun_out/trasr.log 2>&1 || exit 1
F=$(ls gpurun_out/trasr/*kernel_trace.csv gpurun_out/trasr/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/prof_step.py $F > gpurun_out/stepasr.txt || exit 1
cat gpurun_out/stepasr.txt
