#!/bin/bash
# the same default model timed back to back in one process (per-model stream placement),
# third stream at high priority (default) and at normal priority
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 scripts/ab_flags.py - - - 2>&1 | grep -v amdgpu.ids
MOG_S3_HIGH=0 timeout -k 10 300 python3 scripts/ab_flags.py - - - 2>&1 | grep -v amdgpu.ids
