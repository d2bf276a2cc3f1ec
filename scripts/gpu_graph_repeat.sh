#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 scripts/graph_bf16_repeat.py bf16 10 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python3 scripts/graph_bf16_repeat.py fp32 6 2>&1 | grep -v amdgpu.ids
