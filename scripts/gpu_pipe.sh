#!/bin/bash
# pipelined fused-step kernel: parity tests, then timing against the lockstep form
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipe.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pipe_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/vs_pipe_time.py > gpurun_out/pipe_time.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_c64.py tests/test_gpu_torch_ops.py tests/test_gpu_batched_vae.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fused_tests.log 2>&1
