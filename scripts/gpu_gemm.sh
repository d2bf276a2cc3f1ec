#!/bin/bash
# fp32 GEMM iteration: GPU tests, weight-gradient sweeps (64 / 128 tiles), train-step shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gputest.log 2>&1 || exit $?
timeout -k 10 120 env MOG_GEMM_TILE=64 SPLITS=4,8,16,32,48 python scripts/sweep_dw.py > gpurun_out/sweep64.log 2>&1 || exit $?
timeout -k 10 120 env MOG_GEMM_TILE=128 SPLITS=4,8,16,32,48 python scripts/sweep_dw.py > gpurun_out/sweep128.log 2>&1 || exit $?
timeout -k 10 120 python scripts/bench_gemm_f32.py > gpurun_out/gemm_auto.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench.log 2>&1
