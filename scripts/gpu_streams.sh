#!/bin/bash
# The GPU suite (incl. the stream-ordering tests) and one pass of the bf16 /
# fp32 batch-64 determinism probe.
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r05_gputest.log 2>&1 &&
timeout -k 10 300 python -u scripts/bf16_b64_determinism.py bf16 300 > gpurun_out/r05_det.log 2>&1 &&
timeout -k 10 300 python -u scripts/bf16_b64_determinism.py fp32 150 >> gpurun_out/r05_det.log 2>&1
rc=$?
tail -15 gpurun_out/r05_gputest.log; cat gpurun_out/r05_det.log 2>/dev/null | grep -v amdgpu.ids
exit $rc
