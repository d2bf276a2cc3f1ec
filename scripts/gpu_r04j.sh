#!/bin/bash
# tests after the serialized-load fixes, then SQ counters of the x3 GEMMs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_parity.py tests/test_gpu_batched_vae.py tests/test_gpu_asr.py tests/test_gpu_graph.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04j_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r04j_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/r04j_tests.log | head
[ $rc -le 1 ] || exit $rc
bash scripts/pmc_x3.sh
bash scripts/gpu_r04k.sh
