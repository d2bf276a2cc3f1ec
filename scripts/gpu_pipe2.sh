#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u scripts/vs_pipe_phases.py > gpurun_out/pipe_phases.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/vs_pipe_phases.py prio > gpurun_out/pipe_prio.log 2>&1
