#!/bin/bash
# fused-step iteration: bf16 / fused GPU tests, then the bench (fused-step roofline lines)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_c64.py tests/test_gpu_torch_ops.py tests/test_gpu_batched_vae.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gputest_vs.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench.log 2>&1 || exit $?
MOG_VS_TIMING=1 timeout -k 10 120 python scripts/vs_once.py > gpurun_out/vs_timing.log 2>&1
