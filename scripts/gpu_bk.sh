#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python scripts/bench_gemm_f32.py > gpurun_out/gemm_bk16.log 2>&1 || exit $?
MOG_GEMM_BK=32 timeout -k 10 120 python scripts/bench_gemm_f32.py > gpurun_out/gemm_bk32.log 2>&1 || exit $?
MOG_GEMM_BK=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gputest_bk32.log 2>&1 || exit $?
MOG_GEMM_BK=32 timeout -k 10 200 python bench.py --extras 0 --cpu-baseline 0 > gpurun_out/bench_bk32.log 2>&1
timeout -k 10 120 python scripts/host_profile.py 64 30 > gpurun_out/hostprof.log 2>&1
