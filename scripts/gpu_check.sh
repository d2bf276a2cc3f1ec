#!/bin/bash
# full GPU tests, the default bench (no CPU leg), host-side profile at B = 64
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gputest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 120 python scripts/host_profile.py 64 30 > gpurun_out/hostprof.log 2>&1
