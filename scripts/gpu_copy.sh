#!/bin/bash
mkdir -p gpurun_out
for v in 0 1 2 3 4 5; do
  timeout -k 10 60 env MOG_COPY_VARIANT=$v python -u scripts/copy_bw.py >> gpurun_out/copy.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/copy.log
