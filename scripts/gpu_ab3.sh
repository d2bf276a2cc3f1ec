#!/bin/bash
# A/B: side-stream VAE weight gradients forked before / after the STN read backward
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in 0 1 0 1; do
  MOG_SIDE_AFTER_READ=$v timeout -k 10 200 python bench.py --extras 0 --cpu-baseline 0 --roofline-batch 0 --steps 30 > gpurun_out/ab3_$v.log 2>&1 || exit $?
  echo "side_after_read=$v $(tail -1 gpurun_out/ab3_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3))')"
done
