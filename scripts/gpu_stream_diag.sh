#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u ${SCRIPT:-scripts/stream_diag2.py} ${ARGS:-air fp32 1024} > gpurun_out/r05_sdiag.log 2>&1
rc=$?; cat gpurun_out/r05_sdiag.log | grep -v amdgpu.ids; exit $rc
