#!/bin/bash
# fp32 train step with the side stream CU-masked (MOG_SIDE_CU_RESERVE)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in 0 16 32 64 0 32; do
  MOG_SIDE_CU_RESERVE=$r timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 --extras 0 --roofline-batch 0 > gpurun_out/r04k_$r.log 2>&1 || { tail -3 gpurun_out/r04k_$r.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/r04k_$r.log').read().strip().splitlines()[-1]);print('reserve $r: fp32 step', round(d['ms_per_step'],3), 'ms')"
done
