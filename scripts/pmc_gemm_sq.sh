#!/bin/bash
# SQ stall counters of the fp32 GEMM micro-benchmark (one --pmc pass per
# variant; GRBM clock for the effective-clock estimate).
# usage: bash scripts/pmc_gemm_sq.sh "<shapes>" "<env assignments per variant>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp GEMM_ONLY="${1:-xproj,enc2,enc1}"
shift
i=0
for v in "${@:-X=0}"; do
  rm -rf gpurun_out/pmc_sq$i
  env $v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d gpurun_out/pmc_sq$i -o run -- python3 scripts/bench_gemm_f32.py > gpurun_out/pmc_sq$i.log 2>&1 || exit 1
  i=$((i + 1))
done
