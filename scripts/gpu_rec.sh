#!/bin/bash
# one GPU: recurrent-rows weight gradient on the side stream (1) or main (0); GPU suites
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for p in fp32 bf16; do
for v in 0 1 0 1; do
  MOG_REC_SIDE=$v timeout -k 10 200 python bench.py --precision $p --extras 0 --cpu-baseline 0 --roofline-batch 0 --steps 30 > gpurun_out/rec_${p}_$v.log 2>&1 || exit $?
  echo "$p rec_side=$v $(tail -1 gpurun_out/rec_${p}_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3))')"
done
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/rec_tests.log 2>&1 || { tail -30 gpurun_out/rec_tests.log; exit 1; }
tail -1 gpurun_out/rec_tests.log
