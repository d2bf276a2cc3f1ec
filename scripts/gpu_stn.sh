#!/bin/bash
# STN backward iteration: GPU tests that exercise it, the micro-benchmark, then the step traces
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_c64.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gputest_stn.log 2>&1 || exit $?
timeout -k 10 120 python scripts/bench_stn.py 24576 > gpurun_out/stn.log 2>&1 || exit $?
bash scripts/gpu_trace.sh
