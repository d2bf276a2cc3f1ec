#!/bin/bash
# small weight-gradient GEMMs (split-K target sweep), then the GEMM tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
MOG_AIR_LIB=mog-asr_amd/build_ab/libmog_air.so timeout -k 10 120 python3 scripts/x3nt_bench.py > gpurun_out/x3nt_old.log 2>&1 || { tail -5 gpurun_out/x3nt_old.log; exit 1; }
grep NT gpurun_out/x3nt_old.log
timeout -k 10 120 python3 scripts/x3nt_bench.py > gpurun_out/x3nt_new.log 2>&1 || { tail -5 gpurun_out/x3nt_new.log; exit 1; }
grep NT gpurun_out/x3nt_new.log
timeout -k 10 120 python3 scripts/dw_small_bench.py > gpurun_out/dw_small.log 2>&1 || { tail -5 gpurun_out/dw_small.log; exit 1; }
grep -v amdgpu.ids gpurun_out/dw_small.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/x3nt_tests.log 2>&1; tail -2 gpurun_out/x3nt_tests.log
bash scripts/pmc_x3nt.sh
