#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_x3.py tests/test_gpu_asr.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04g_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r04g_tests.log
[ $rc -le 1 ] || exit $rc; grep -E "^(FAILED|ERROR)" gpurun_out/r04g_tests.log | head -10
timeout -k 10 200 python -u -c "
import sys; sys.path[:0]=['.','mog-asr_amd']
import torch, bench
dev=torch.device('cuda:0')
for prec in ('fp32','bf16'):
    el, m = bench.timed_train(prec, 8192, 10, 3, dev, model=bench.make_asr_model(prec, dev, 'asr_'+prec))
    print('ASR', prec, round(el/10*1e3,3), 'ms')
el, m = bench.timed_train('bf16', 8192, 10, 3, dev, scope='b16ev', events=False)
print('AIR bf16 no events', round(el/10*1e3,3), 'ms')
el, m = bench.timed_train('bf16', 8192, 10, 3, dev, scope='b16ev2', events=True)
print('AIR bf16 events', round(el/10*1e3,3), 'ms')
" 2>&1 | grep -v amdgpu.ids
rm -rf gpurun_out/trasr
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trasr -o run -- python3 scripts/asr_steps.py > gpurun_out/trasr.log 2>&1 || { tail -3 gpurun_out/trasr.log; exit 1; }
echo "asr trace ok"
