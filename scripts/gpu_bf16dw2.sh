#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 120 python bench.py --precision bf16 --extras 0 --cpu-baseline 0 --steps 30 > gpurun_out/bfdw.log 2>&1 || exit $?
  echo "$* $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bfdw.log)"
}
run MOG_DW_TARGET=256
run MOG_DW_TARGET=512
run MOG_DW_TARGET=1024
run MOG_DW_TARGET=2048
run MOG_DW_TARGET=256
