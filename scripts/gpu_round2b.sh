#!/bin/bash
# GPU session script: tests, bench, fp32 weight-gradient split-K / tile sweep
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gputest.log 2>&1 || exit $?
timeout -k 10 120 env MOG_GEMM_TILE=64 python scripts/sweep_dw.py > gpurun_out/sweep64.log 2>&1 || exit $?
timeout -k 10 120 env MOG_GEMM_TILE=128 python scripts/sweep_dw.py > gpurun_out/sweep128.log 2>&1 || exit $?
timeout -k 10 120 python scripts/bench_gemm_f32.py ref > gpurun_out/gemm_ref.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
