#!/bin/bash
# split-K target of the fp32 weight gradients (side stream) vs train-step time
set -o pipefail
mkdir -p gpurun_out
for t in 2048 512 1024 4096 2048; do
  MOG_DW32_TARGET=$t timeout -k 10 120 python bench.py --extras 0 --cpu-baseline 0 --steps 30 > gpurun_out/dwt_$t.log 2>&1 || exit $?
  echo "target $t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dwt_$t.log)"
done
