#!/bin/bash
# A/B of two builds of libmog_air.so (the in-tree one and ALT) on the fused
# step kernel (scripts/vs_time.py) and the train step (bench extras off).
mkdir -p gpurun_out
ALT=${ALT:-mog-asr_amd/build_alt/libmog_air.so}
for i in 1 2; do
  timeout -k 10 120 python -u scripts/vs_time.py 65536 >> gpurun_out/ab_lib.log 2>&1 || exit 1
  timeout -k 10 120 env MOG_AIR_LIB=$ALT python -u scripts/vs_time.py 65536 | sed 's/^/ALT /' >> gpurun_out/ab_lib.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/ab_lib.log
