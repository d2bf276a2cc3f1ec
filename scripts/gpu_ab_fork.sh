#!/bin/bash
# fp32 step: weight-gradient fork before vs after the STN read backward
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for f in 0 1 0 1; do
  MOG_FORK_AFTER_READ=$f timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 --extras 0 --roofline-batch 0 > gpurun_out/abfork_$f.log 2>&1 || { tail -3 gpurun_out/abfork_$f.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/abfork_$f.log').read().strip().splitlines()[-1]);print('fork_after_read $f: fp32 step', round(d['ms_per_step'],3), 'ms')"
done
