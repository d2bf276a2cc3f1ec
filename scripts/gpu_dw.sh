#!/bin/bash
# weight-gradient GEMM shapes under the tile variants
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
: > gpurun_out/dw.log
for v in "" "MOG_GEMM_TILE=128" "MOG_GEMM_BK=16" "MOG_GEMM_TILE=12864"; do
  echo "== $v" >> gpurun_out/dw.log
  env $v timeout -k 10 120 python -u scripts/dw_bench.py 256 512 1024 2048 >> gpurun_out/dw.log 2>&1 || exit $?
done
