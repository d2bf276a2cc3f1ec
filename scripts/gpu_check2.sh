#!/bin/bash
# full GPU tests, the default bench (no CPU leg), a kernel trace of the headline step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gputest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench.log 2>&1 || exit $?
rm -rf gpurun_out/tr8192
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr8192 -o run -- python3 bench.py --steps 6 --warmup 2 --cpu-baseline 0 --extras 0 --roofline-batch 0 --batch 8192 > gpurun_out/tr8192.log 2>&1 || exit 1
python3 scripts/prof_step.py gpurun_out/tr8192/run_kernel_trace.csv > gpurun_out/step8192.txt
