#!/bin/bash
# x3 weight-gradient GEMM: accuracy tests, then the fp32 step with the x-part gradient on
# the fp32 chain (x3=0) and on x3 at split-K 4 / 8 / 16, then the GPU suites
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_x3.py > gpurun_out/x3_tests.log 2>&1 || { tail -40 gpurun_out/x3_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/x3_tests.log | tail -12
for cfg in "0 8" "1 4" "1 8" "1 16" "0 8" "1 8"; do
  set -- $cfg
  MOG_X_GRAD_X3=$1 MOG_X3_SPLITK=$2 timeout -k 10 200 python bench.py --extras 0 --cpu-baseline 0 --roofline-batch 0 --steps 30 > gpurun_out/x3_b_$1_$2.log 2>&1 || exit $?
  echo "x3=$1 splitk=$2 $(tail -1 gpurun_out/x3_b_$1_$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3))')"
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/x3_all.log 2>&1 || { tail -30 gpurun_out/x3_all.log; exit 1; }
tail -2 gpurun_out/x3_all.log
