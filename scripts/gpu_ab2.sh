#!/bin/bash
# A/B of library builds (scripts/bin/libmog_air_<name>.so) on the fused step kernel
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
: > gpurun_out/ab.log
for i in 1 2; do
  for n in "$@"; do
    echo "== $n" >> gpurun_out/ab.log
    MOG_AIR_LIB=$PWD/scripts/bin/libmog_air_$n.so timeout -k 10 120 python -u scripts/vs_variants.py 65536 50 MOG_VS_PIPE=0 MOG_VS_PIPE=0 MOG_VS_PIPE=0,MOG_VS_LA=5 MOG_VS_PIPE=0:timing >> gpurun_out/ab.log 2>&1 || exit $?
  done
done
