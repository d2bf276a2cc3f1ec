#!/bin/bash
# bf16 configuration: x-rows gradient on the one-piece x3p kernel vs gemm_bf16; GPU suites
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in 0 1 0 1; do
  MOG_X_GRAD_BF16_X1=$v timeout -k 10 200 python bench.py --precision bf16 --extras 0 --cpu-baseline 0 --roofline-batch 0 --steps 30 > gpurun_out/x1_$v.log 2>&1 || exit $?
  echo "bf16 x1=$v $(tail -1 gpurun_out/x1_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3))')"
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/x1_tests.log 2>&1 || { tail -30 gpurun_out/x1_tests.log; exit 1; }
tail -1 gpurun_out/x1_tests.log
