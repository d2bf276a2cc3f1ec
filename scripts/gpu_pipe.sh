#!/bin/bash
# pipelined fused step: bitwise tests, then lockstep vs pipelined launch times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_pipe.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pipe_test.log 2>&1; rc=$?
tail -15 gpurun_out/pipe_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/vs_pipe_time.py > gpurun_out/pipe_time.log 2>&1 || { tail -20 gpurun_out/pipe_time.log; exit 1; }
cat gpurun_out/pipe_time.log
MOG_VS_TIMING=1 MOG_VS_PIPE=1 timeout -k 10 120 python -u -c "
import os,sys; sys.path[:0]=['.','mog-asr_amd']
import torch, bench
bench.fused_step_roofline(65536, 3, torch.device('cuda:0'))
" 2>&1 | grep -i "phases\|pipe" | tail -4
