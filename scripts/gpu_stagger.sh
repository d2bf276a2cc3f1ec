#!/bin/bash
# fused bf16 step: stagger half of the first-round workgroups (MOG_VS_STAGGER ticks of 10 ns)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for st in 0 2500 5000 7500 0 5000; do
  MOG_VS_STAGGER=$st timeout -k 10 100 python3 -u scripts/vs_time.py 65536 > gpurun_out/st_$st.log 2>&1 || exit $?
  echo "stagger $st: $(tail -1 gpurun_out/st_$st.log)"
done
