#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
MOG_X3_STAGES=1 timeout -k 10 120 python scripts/x3_time.py || exit $?
MOG_X3_STAGES=2 timeout -k 10 120 python scripts/x3_time.py || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_x3.py > gpurun_out/x3b_tests.log 2>&1 || { tail -40 gpurun_out/x3b_tests.log; exit 1; }
tail -1 gpurun_out/x3b_tests.log
for cfg in "0 8" "1 8" "0 8" "1 8"; do
  set -- $cfg
  MOG_X_GRAD_X3=$1 MOG_X3_SPLITK=$2 timeout -k 10 200 python bench.py --extras 0 --cpu-baseline 0 --roofline-batch 0 --steps 30 > gpurun_out/x3b_$1_$2.log 2>&1 || exit $?
  echo "x3=$1 splitk=$2 $(tail -1 gpurun_out/x3b_$1_$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3))')"
done
