#!/bin/bash
# NT x3 prefetch distance 1 vs 2 (after the load fixes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for pd in 1 2; do
  MOG_X3NT_PD=$pd timeout -k 10 120 python3 scripts/x3nt_bench.py > gpurun_out/x3nt_pd$pd.log 2>&1 || { tail -5 gpurun_out/x3nt_pd$pd.log; exit 1; }
  grep NT gpurun_out/x3nt_pd$pd.log
done
