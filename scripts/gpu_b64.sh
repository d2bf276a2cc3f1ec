#!/bin/bash
# kernel list of the captured batch-64 fp32 step (prof_step's per-kernel sums)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
rm -rf gpurun_out/trg64
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trg64 -o run -- python3 scripts/b64_graph_trace.py 64 ${WHICH:-} > gpurun_out/trg64.log 2>&1 || { tail -3 gpurun_out/trg64.log; exit 1; }
grep "ms/step" gpurun_out/trg64.log
f=$(ls gpurun_out/trg64/*kernel_trace.csv gpurun_out/trg64/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/prof_step.py "$f" > gpurun_out/step64g.txt && cat gpurun_out/step64g.txt
python3 scripts/step_timeline.py "$f" > gpurun_out/step64g_timeline.txt
