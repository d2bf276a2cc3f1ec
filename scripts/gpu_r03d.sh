#!/bin/bash
# captured train step: parity tests, batch-64 bench (graph vs eager); fp32 fused phases
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_torch_ops.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/graphtest.log 2>&1 || { tail -40 gpurun_out/graphtest.log; exit 1; }
tail -2 gpurun_out/graphtest.log
timeout -k 10 200 python -u bench.py --batch 64 --steps 50 --warmup 5 --extras 0 --cpu-baseline 0 --roofline-batch 0 > gpurun_out/b64.log 2>&1 || exit $?
tail -1 gpurun_out/b64.log | cut -c1-300
timeout -k 10 200 python -u -c "
import sys, torch; sys.path.insert(0, 'mog-asr_amd'); sys.path.insert(0, '.')
import bench
dev = torch.device('cuda:0')
for B in (64, 256, 1024):
    for g in (False, True):
        el, m = bench.timed_train('fp32', B, 30, 5, dev, scope='g%d%d' % (B, g), graph=g)
        print(f'B={B} graph={g}: {el / 30 * 1e3:.3f} ms/step', flush=True)
" > gpurun_out/graph_b.log 2>&1 || exit $?
cat gpurun_out/graph_b.log
timeout -k 10 200 python -u scripts/f32_time.py 24576 > gpurun_out/f32_time.log 2>&1 || exit $?
cat gpurun_out/f32_time.log
