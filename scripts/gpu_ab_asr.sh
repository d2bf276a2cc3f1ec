#!/bin/bash
# ASR step: weight gradients per loop step on the side stream vs after the loop (fp32, bf16),
# then the ASR GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 scripts/ab_asr.py bf16 - HEADS_S3=0 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python3 scripts/ab_asr.py fp32 - HEADS_S3=0 2>&1 | grep -v amdgpu.ids
timeout -k 10 400 python -u -m pytest tests/test_gpu_asr.py tests/test_gpu_x3.py tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/asr_tests.log 2>&1; rc=$?
tail -2 gpurun_out/asr_tests.log; exit $rc
