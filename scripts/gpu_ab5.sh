#!/bin/bash
# noise + resets on the side stream under the x-projection: fp32 / bf16 / graphed b64 bench,
# then the GPU suites that exercise the noise (parity, graph, fused, bf16, DP, ASR)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for p in fp32 bf16; do
  timeout -k 10 200 python bench.py --precision $p --extras 0 --cpu-baseline 0 --roofline-batch 0 --steps 30 > gpurun_out/ab5_${p}.log 2>&1 || exit $?
  echo "$p $(tail -1 gpurun_out/ab5_${p}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3))')"
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/ab5_tests.log 2>&1 || { tail -30 gpurun_out/ab5_tests.log; exit 1; }
tail -2 gpurun_out/ab5_tests.log
