#!/bin/bash
# The default bench line (driver contract) into gpurun_out/${TAG:-r05}_bench.log
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG:-r05}_bench.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/${TAG:-r05}_bench.log | tail -c 6000
exit $rc
