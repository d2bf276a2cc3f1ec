#!/bin/bash
# fused-step parity (lockstep form) then variant timings
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "pipe or fused" > gpurun_out/fused_parity.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/vs_variants.py "$@" > gpurun_out/vs_var.log 2>&1
