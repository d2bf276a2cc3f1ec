#!/bin/bash
# optimizer / step-kernel changes: parity + batch-64 timing + a kernel trace of the captured step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_graph.py tests/test_gpu_torch_ops.py tests/test_gpu_batched_vae.py tests/test_gpu_asr.py tests/test_gpu_dp.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/small2.log 2>&1 || { tail -30 gpurun_out/small2.log; exit 1; }
tail -1 gpurun_out/small2.log
timeout -k 10 200 python -u -c "
import sys, torch; sys.path.insert(0, 'mog-asr_amd'); sys.path.insert(0, '.')
import bench
dev = torch.device('cuda:0')
for B in (64, 8192):
    for g in (False, True):
        el, m = bench.timed_train('fp32', B, 20, 5, dev, scope='s%d%d' % (B, g), graph=g)
        print(f'B={B} graph={g}: {el / 20 * 1e3:.3f} ms/step', flush=True)
" > gpurun_out/small2_b.log 2>&1 || exit $?
cat gpurun_out/small2_b.log
rm -rf gpurun_out/trg64
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trg64 -o run -- python3 scripts/b64_graph_trace.py 64 > gpurun_out/trg64.log 2>&1 || exit 1
python3 scripts/prof_step.py $(ls gpurun_out/trg64/*kernel_trace.csv gpurun_out/trg64/*/*kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/step64g.txt || exit 1
cat gpurun_out/step64g.txt
