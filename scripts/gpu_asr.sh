#!/bin/bash
# ASR: bit-exact suites (incl. the fused fp32 step per loop step) + configs[2] step times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_asr.py tests/test_gpu_dp.py tests/test_gpu_torch_ops.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/asr.log 2>&1 || { tail -30 gpurun_out/asr.log; exit 1; }
tail -1 gpurun_out/asr.log
timeout -k 10 300 python -u -c "
import sys, torch; sys.path.insert(0, 'mog-asr_amd'); sys.path.insert(0, '.')
import bench
dev = torch.device('cuda:0')
for prec in ('fp32', 'bf16'):
    el, m = bench.timed_train(prec, 8192, 10, 3, dev, model=bench.make_asr_model(prec, dev, 'a' + prec))
    print(f'ASR {prec} B=8192: {el / 10 * 1e3:.3f} ms/step', flush=True)
el, m = bench.timed_train('fp32', 64, 30, 5, dev, model=bench.make_asr_model('fp32', dev, 'a64'))
print(f'ASR fp32 B=64: {el / 30 * 1e3:.3f} ms/step', flush=True)
" > gpurun_out/asr_b.log 2>&1 || exit $?
cat gpurun_out/asr_b.log
