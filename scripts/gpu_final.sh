#!/bin/bash
# round-end rehearsal: GPU tests, smoke(), default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/final_tests.log 2>&1 || { tail -30 gpurun_out/final_tests.log; exit 1; }
tail -1 gpurun_out/final_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/final_bench.log 2>&1 || { tail -20 gpurun_out/final_bench.log; exit 1; }
tail -1 gpurun_out/final_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('headline', round(d['ms_per_step'],3), 'b64', round(d['config_1_batch64_fp32']['ms_per_step'],3), d['config_1_batch64_fp32']['eager_ms_per_step'], 'bf16', round(d['configs_1_bf16']['ms_per_step'],3))"
