#!/bin/bash
# fp32 fused step: parity tests, then fused vs unfused timing + phases
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_f32.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/f32_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u scripts/f32_time.py 65536 > gpurun_out/f32_time.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/f32_time.py 24576 >> gpurun_out/f32_time.log 2>&1 || exit $?
