#!/bin/bash
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pwg
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pwg/kt -o run -- python3 $R/scripts/wgrad_shapes.py > $R/gpurun_out/pwg/kt.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES -d $R/gpurun_out/pwg/p1 -o run -- python3 $R/scripts/wgrad_shapes.py > $R/gpurun_out/pwg/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/pwg/p2 -o run -- python3 $R/scripts/wgrad_shapes.py > $R/gpurun_out/pwg/p2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max TD_BUSY_avr -d $R/gpurun_out/pwg/p3 -o run -- python3 $R/scripts/wgrad_shapes.py > $R/gpurun_out/pwg/p3.log 2>&1 || exit 1
