#!/bin/bash
# per-tile phase times of the lockstep fused kernel (MOG_VS_TIMING) and the
# fp32 fused kernel, at the roofline shapes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
MOG_VS_TIMING=1 timeout -k 10 120 python3 scripts/vs_time.py 65536 > gpurun_out/vsph.log 2>&1 || { tail -3 gpurun_out/vsph.log; exit 1; }
grep -v amdgpu.ids gpurun_out/vsph.log | tail -6
MOG_VS_TIMING=1 timeout -k 10 120 python3 scripts/f32_time.py > gpurun_out/f32ph.log 2>&1 || { tail -3 gpurun_out/f32ph.log; exit 1; }
grep -v amdgpu.ids gpurun_out/f32ph.log | tail -6
