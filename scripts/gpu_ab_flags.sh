#!/bin/bash
# AIRModel flag A/B over the bench's fp32 / bf16 / dSprites train steps (scripts/ab_flags.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 scripts/ab_flags.py "$@" 2>&1 | grep -v amdgpu.ids
