#!/bin/bash
# full GPU suite + A/B of the x3 input gradients + LA sweep + the default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04d_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04d_tests.log
[ $rc -le 1 ] || exit $rc; grep -E "^(FAILED|ERROR)" gpurun_out/r04d_tests.log | head -20
for i in 1 2; do for v in 0 1; do
  MOG_VAE_DX_X3=$v timeout -k 10 120 python bench.py --extras 0 --cpu-baseline 0 > gpurun_out/r04d_ab_$v.log 2>&1 || { tail -5 gpurun_out/r04d_ab_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r04d_ab_$v.log').read().strip().splitlines()[-1]); print('VAE_DX_X3=$v', round(d['ms_per_step'],3), 'ms')"
done; done
for la in 3 4 5; do
MOG_VS_LA=$la timeout -k 10 120 python -u -c "
import os,sys; sys.path[:0]=['.','mog-asr_amd']
import torch, bench
r = bench.fused_step_roofline(65536, 20, torch.device('cuda:0'))
print('LA=$la', round(r['avg_launch_us'],1), 'us', round(r['frac'],3))
" 2>&1 | grep LA
done
timeout -k 10 500 python bench.py > gpurun_out/r04d_bench.log 2>&1 || { tail -5 gpurun_out/r04d_bench.log; exit 1; }
tail -1 gpurun_out/r04d_bench.log | cut -c1-1500
