#!/bin/bash
# host issue cost of the captured batch-64 step, by part (scripts/graph_host_time.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
timeout -k 10 200 python3 scripts/graph_host_time.py 64 2>&1 | grep -v amdgpu.ids
