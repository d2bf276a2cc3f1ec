#!/bin/bash
# ASR fp32 step: the VAE input gradients at 8,192 rows per step on the NT x3
# form vs the fp32 GEMM (MOG_X3_DX_MIN_ROWS), and the AIR fp32 step unchanged
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for r in 16384 8192 16384 8192; do
  MOG_X3_DX_MIN_ROWS=$r timeout -k 10 200 python3 -c "
import sys; sys.path[:0]=['.','mog-asr_amd']
import torch, bench
dev=torch.device('cuda:0')
el, m = bench.timed_train('fp32', 8192, 10, 3, dev, model=bench.make_asr_model('fp32', dev, 'asr_ab'))
print('min_rows $r: ASR fp32', round(el/10*1e3,3), 'ms')
" 2>&1 | grep ASR
done
