#!/bin/bash
# captured batch-64 fp32 step with 2- vs 4-stage small-M GEMMs, and the bit-exact GEMM tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for ns in 2 4 2 4; do
  MOG_GEMM_SMALL_NS=$ns timeout -k 10 120 python3 scripts/b64_graph_trace.py 64 > gpurun_out/b64ns_$ns.log 2>&1 || { tail -3 gpurun_out/b64ns_$ns.log; exit 1; }
  echo "ns=$ns $(grep ms/step gpurun_out/b64ns_$ns.log)"
done
MOG_GEMM_SMALL_NS=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_graph.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/b64ns_tests.log 2>&1; tail -2 gpurun_out/b64ns_tests.log
