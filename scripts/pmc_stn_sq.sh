#!/bin/bash
# SQ instruction-mix / stall counters of the STN kernels (scripts/bench_stn.py
# at B rows), one --pmc pass per counter set.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=${1:-24576}
rm -rf gpurun_out/pmc_stn1 gpurun_out/pmc_stn2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  --output-format csv -d gpurun_out/pmc_stn1 -o run -- python3 scripts/bench_stn.py $B wbwd > gpurun_out/pmc_stn1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_stn2 -o run -- python3 scripts/bench_stn.py $B wbwd > gpurun_out/pmc_stn2.log 2>&1 || exit 1
