#!/bin/bash
# fused bf16 step: 64-image vs 32-image tiles at the train step's T*B rows
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for mt in 4 3; do
  MOG_VS_MT=$mt timeout -k 10 100 python3 -u scripts/vs_time.py 24576 > gpurun_out/mt_$mt.log 2>&1 || exit $?
  tail -1 gpurun_out/mt_$mt.log
done
for mt in 4 3; do
  MOG_VS_MT=$mt timeout -k 10 200 python bench.py --precision bf16 --extras 0 --cpu-baseline 0 --roofline-batch 0 --steps 20 > gpurun_out/mtb_$mt.log 2>&1 || exit $?
  echo "MT=$mt bf16 step $(tail -1 gpurun_out/mtb_$mt.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3))') ms"
done
