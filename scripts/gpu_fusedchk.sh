#!/bin/bash
# fused-step parity tests + timing after a change to vae_step.hip
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_c64.py tests/test_gpu_fused_f32.py tests/test_gpu_torch_ops.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fusedchk.log 2>&1 || { tail -30 gpurun_out/fusedchk.log; exit 1; }
tail -2 gpurun_out/fusedchk.log
timeout -k 10 200 python3 -u scripts/vs_phases.py 65536 timing > gpurun_out/vsdiag_t31.log 2>&1 || exit $?
cat gpurun_out/vsdiag_t31.log
timeout -k 10 200 python3 -u scripts/vs_time.py 65536 > gpurun_out/vs_time.log 2>&1 || exit $?
timeout -k 10 200 python3 -u scripts/vs_time.py 65536 64 >> gpurun_out/vs_time.log 2>&1 || exit $?
cat gpurun_out/vs_time.log
