#!/bin/bash
# run one python script on the GPU box: OUT=<log name> bash scripts/gpu_run.sh script.py args
mkdir -p gpurun_out
timeout -k 10 ${LIMIT:-300} python -u "$@" > gpurun_out/${OUT:-run}.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/${OUT:-run}.log | tail -40
exit $rc
