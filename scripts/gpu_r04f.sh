#!/bin/bash
# A/B: high-priority main stream x weight-gradient split-K target
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for i in 1 2; do for pr in 0 1; do for tg in 2048 512; do
  MOG_MAIN_PRIO=$pr MOG_DW32_TARGET=$tg timeout -k 10 120 python bench.py --extras 0 --cpu-baseline 0 > gpurun_out/r04f_$pr$tg.log 2>&1 || { tail -5 gpurun_out/r04f_$pr$tg.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r04f_$pr$tg.log').read().strip().splitlines()[-1]); print('prio=$pr dw_target=$tg', round(d['ms_per_step'],3), 'ms')"
done; done; done
