#!/bin/bash
# SQ stall counters of the x3 GEMMs (NT and both TN forms) at the fp32 step's
# shapes, one --pmc pass, summarised per kernel and grid (scripts/pmc_sq_table.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_x3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_x3 -o run -- python3 scripts/x3_lib_bench.py > gpurun_out/pmc_x3.log 2>&1 || { tail -3 gpurun_out/pmc_x3.log; exit 1; }
python3 scripts/pmc_sq_table.py gpurun_out/pmc_x3
