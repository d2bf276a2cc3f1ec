#!/bin/bash
# small-M GEMM tiles: bit-exact parity suites at small batches + batch-64 step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_batched_vae.py tests/test_gpu_graph.py tests/test_gpu_fused_f32.py tests/test_gpu_asr.py tests/test_gpu_torch_ops.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/small.log 2>&1 || { tail -30 gpurun_out/small.log; exit 1; }
tail -1 gpurun_out/small.log
timeout -k 10 200 python -u -c "
import sys, torch; sys.path.insert(0, 'mog-asr_amd'); sys.path.insert(0, '.')
import bench
dev = torch.device('cuda:0')
for B in (64, 256):
    for g in (False, True):
        el, m = bench.timed_train('fp32', B, 30, 5, dev, scope='s%d%d' % (B, g), graph=g)
        print(f'B={B} graph={g}: {el / 30 * 1e3:.3f} ms/step', flush=True)
" > gpurun_out/small_b.log 2>&1 || exit $?
cat gpurun_out/small_b.log
