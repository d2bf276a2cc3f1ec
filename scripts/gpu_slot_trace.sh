#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
rm -rf gpurun_out/slot
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/slot -o run -- python3 scripts/slot_trace.py 3 > gpurun_out/slot.log 2>&1 || { tail -3 gpurun_out/slot.log; exit 1; }
grep -A1 "ms/step" gpurun_out/slot.log
f=$(ls gpurun_out/slot/*kernel_trace.csv gpurun_out/slot/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/slot_compare.py "$f" > gpurun_out/slot_cmp.txt && head -30 gpurun_out/slot_cmp.txt
