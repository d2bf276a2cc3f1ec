#!/bin/bash
# kernel traces of the headline step at B = 8192 and B = 64 (idle-gap analysis)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in 8192 64; do
  rm -rf gpurun_out/tr$B
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr$B -o run -- python3 bench.py --steps 6 --warmup 2 --cpu-baseline 0 --extras 0 --roofline-batch 0 --batch $B > gpurun_out/tr$B.log 2>&1 || exit 1
  python3 scripts/prof_step.py $(ls gpurun_out/tr$B/*kernel_trace.csv gpurun_out/tr$B/*/*kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/step$B.txt || exit 1
done
