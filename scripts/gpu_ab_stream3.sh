#!/bin/bash
# fp32 step: the recurrent rows gradient on the side stream vs the third stream (MOG_REC_STREAM3;
# the heads gradients measured the same way with MOG_HEADS_STREAM3)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for f in 0 1 0 1; do
  MOG_REC_STREAM3=$f timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 --extras 0 --roofline-batch 0 > gpurun_out/abs3_$f.log 2>&1 || { tail -3 gpurun_out/abs3_$f.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/abs3_$f.log').read().strip().splitlines()[-1]);print('rec_stream3 $f: fp32 step', round(d['ms_per_step'],3), 'ms')"
done
MOG_REC_STREAM3=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/abs3_tests.log 2>&1; tail -1 gpurun_out/abs3_tests.log
