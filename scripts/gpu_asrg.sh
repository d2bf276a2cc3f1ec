#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/asrg.log 2>&1 || { tail -30 gpurun_out/asrg.log; exit 1; }
tail -1 gpurun_out/asrg.log
timeout -k 10 300 python -u -c "
import sys, torch; sys.path.insert(0, 'mog-asr_amd'); sys.path.insert(0, '.')
import bench
dev = torch.device('cuda:0')
for g in (False, True):
    el, m = bench.timed_train('fp32', 64, 30, 5, dev, graph=g, model=bench.make_asr_model('fp32', dev, 'ag%d' % g))
    print(f'ASR fp32 B=64 graph={g}: {el / 30 * 1e3:.3f} ms/step', flush=True)
" > gpurun_out/asrg_b.log 2>&1 || exit $?
cat gpurun_out/asrg_b.log
