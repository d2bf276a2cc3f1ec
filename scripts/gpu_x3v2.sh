#!/bin/bash
# NT x3: single-stage 4-wave form vs the double-buffered 8-wave form
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in 0 1; do
  MOG_X3NT_V2=$v timeout -k 10 120 python3 scripts/x3nt_bench.py > gpurun_out/x3nt_v$v.log 2>&1 || { tail -5 gpurun_out/x3nt_v$v.log; exit 1; }
  sed "s/^/v$v /" gpurun_out/x3nt_v$v.log | grep NT
done
