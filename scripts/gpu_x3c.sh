#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_x3.py > gpurun_out/x3c_tests.log 2>&1 || { tail -40 gpurun_out/x3c_tests.log; exit 1; }
tail -1 gpurun_out/x3c_tests.log
timeout -k 10 120 python scripts/x3_time.py || exit $?
for v in 0 2 0 2; do
  MOG_X_GRAD_X3=$v timeout -k 10 200 python bench.py --extras 0 --cpu-baseline 0 --roofline-batch 0 --steps 30 > gpurun_out/x3c_$v.log 2>&1 || exit $?
  echo "x3=$v $(tail -1 gpurun_out/x3c_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3))')"
done
