#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/stn_concurrency.py none x3_tn bf16_tn x3_nt x3p_tn bf16_nt > gpurun_out/r05_conc4.log 2>&1
rc=$?
grep -hv amdgpu.ids gpurun_out/r05_conc4.log | tail -8
exit $rc
