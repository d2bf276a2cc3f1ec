#!/bin/bash
# measured values behind the loose numeric gates (bf16 ELBO / gradients, ASR bf16 per-tensor)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 MOG_GRAD_REPORT=gpurun_out/asr_grad
timeout -k 10 400 python -u -m pytest -s tests/test_gpu_bf16.py tests/test_gpu_asr.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "vs_fp32_oracle or gradients or elbo or lstm_x" > gpurun_out/gates.log 2>&1 || { tail -30 gpurun_out/gates.log; exit 1; }
grep -E "relative|LSTM kernel|rel_total|passed|failed" gpurun_out/gates.log | cut -c1-300
