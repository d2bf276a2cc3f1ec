#!/bin/bash
# captured batch-64 step with the small-M GEMM pipeline depth MOG_GEMM_SNS = 2 / 3 / 4
# (MOG_GEMM_SNS was a temporary switch, measured and removed: the small-M tiles stay two-stage)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
for n in 2 4 3 2 4 3; do
  echo -n "SNS=$n: "
  MOG_GEMM_SNS=$n timeout -k 10 120 python3 scripts/graph_host_time.py 64 2>&1 | grep "host issue"
done
