#!/bin/bash
# early decoder weight gradients (MOG_WGRAD_EARLY) A/B on the fp32 step, tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for e in 0 1 0 1; do
  MOG_WGRAD_EARLY=$e timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 --extras 0 --roofline-batch 0 > gpurun_out/r04m_$e.log 2>&1 || { tail -3 gpurun_out/r04m_$e.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r04m_$e.log').read().strip().splitlines()[-1]);print('early $e: fp32 step', round(d['ms_per_step'],3), 'ms')"
done
