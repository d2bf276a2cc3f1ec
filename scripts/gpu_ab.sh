#!/bin/bash
# A/B: the fused step kernel of the committed library (scripts/bin/libmog_air_head.so)
# against the working tree's, same box; then the weight-gradient pipeline depths
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
: > gpurun_out/ab.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "fused" > gpurun_out/fused_parity.log 2>&1 || exit $?
for i in 1 2; do
  echo "== head" >> gpurun_out/ab.log
  MOG_AIR_LIB=$PWD/scripts/bin/libmog_air_head.so timeout -k 10 120 python -u scripts/vs_variants.py 65536 50 MOG_VS_PIPE=0,MOG_VS_LA=3 MOG_VS_PIPE=0,MOG_VS_LA=3 MOG_VS_PIPE=0,MOG_VS_LA=5 MOG_VS_PIPE=0:timing >> gpurun_out/ab.log 2>&1 || exit $?
  echo "== tree" >> gpurun_out/ab.log
  timeout -k 10 120 python -u scripts/vs_variants.py 65536 50 MOG_VS_LA=3 MOG_VS_LA=3 MOG_VS_LA=5 MOG_VS_LA=3:timing >> gpurun_out/ab.log 2>&1 || exit $?
done
