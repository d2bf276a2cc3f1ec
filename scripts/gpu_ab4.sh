#!/bin/bash
# A/B: single-GPU heads' weight gradients on the side stream (1) or the main stream (0),
# fp32 headline and bf16; then the graph / fp32 / bf16 GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for p in fp32 bf16; do
for v in 0 1 0 1; do
  MOG_HEADS_SIDE=$v timeout -k 10 200 python bench.py --precision $p --extras 0 --cpu-baseline 0 --roofline-batch 0 --steps 30 > gpurun_out/ab4_${p}_$v.log 2>&1 || exit $?
  echo "$p heads_side=$v $(tail -1 gpurun_out/ab4_${p}_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3))')"
done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_graph.py tests/test_gpu_fused_f32.py tests/test_gpu_bf16.py tests/test_gpu_dp.py > gpurun_out/ab4_tests.log 2>&1 || { tail -30 gpurun_out/ab4_tests.log; exit 1; }
tail -2 gpurun_out/ab4_tests.log
