#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
echo -n "VAE weight gradients on the main stream: "
MOG_VAE_SIDE_SMALL=0 timeout -k 10 300 python3 scripts/bf16_b64_determinism.py bf16 300 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python3 scripts/bf16_b64_determinism.py bf16 300 2>&1 | grep -v amdgpu.ids
