#!/bin/bash
# lockstep vs pipelined (4+4 and 8+8 waves) launch times + per-role phases
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u scripts/vs_pipe_time.py > gpurun_out/pipe_time.log 2>&1 || { tail -20 gpurun_out/pipe_time.log; exit 1; }
cat gpurun_out/pipe_time.log
MOG_AIR_LIB=$PWD/mog-asr_amd/mog_air/_lib_alt/libmog_air.so timeout -k 10 200 python -u scripts/vs_pipe_time.py > gpurun_out/pipe_time8.log 2>&1 || { tail -20 gpurun_out/pipe_time8.log; exit 1; }
echo "8+8:"; cat gpurun_out/pipe_time8.log
for L in "" "$PWD/mog-asr_amd/mog_air/_lib_alt/libmog_air.so"; do
MOG_AIR_LIB=$L MOG_VS_TIMING=1 MOG_VS_PIPE=1 timeout -k 10 120 python -u -c "
import os,sys; sys.path[:0]=['.','mog-asr_amd']
import torch, bench
bench.fused_step_roofline(65536, 3, torch.device('cuda:0'))
" 2>&1 | grep -i "pipe\|detail" | tail -4
done
