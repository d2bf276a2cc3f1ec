#!/bin/bash
# round-4 batch: pipe variants, VAE-weight-gradient x3 A/B, new GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_graph.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04a_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04a_tests.log
[ $rc -le 1 ] || exit $rc; grep -E "^(FAILED|E  )" gpurun_out/r04a_tests.log | head -20
for i in 1 2; do for v in 0 1; do
  MOG_VAE_WGRAD_X3=$v timeout -k 10 120 python bench.py --extras 0 --cpu-baseline 0 > gpurun_out/r04a_ab_$v.log 2>&1 || { tail -5 gpurun_out/r04a_ab_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r04a_ab_$v.log').read().strip().splitlines()[-1]); print('VAE_WGRAD_X3=$v', round(d['ms_per_step'],3), 'ms', d['roofline']['kernel'], round(d['roofline']['frac'],3))"
done; done
bash scripts/gpu_pipe2.sh
