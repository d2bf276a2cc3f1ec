#!/bin/bash
# serialized-load fixes (NT x3 loads/epilogue, gemm_f32 Cin/bias/aux): NT A/B
# against the previous library, GEMM + step tests, fp32 step timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
MOG_AIR_LIB=mog-asr_amd/build_ab/libmog_air.so timeout -k 10 120 python3 scripts/x3nt_bench.py > gpurun_out/x3nt_old.log 2>&1 || { tail -5 gpurun_out/x3nt_old.log; exit 1; }
grep NT gpurun_out/x3nt_old.log
timeout -k 10 120 python3 scripts/x3nt_bench.py > gpurun_out/x3nt_new.log 2>&1 || { tail -5 gpurun_out/x3nt_new.log; exit 1; }
grep NT gpurun_out/x3nt_new.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_fused_f32.py tests/test_gpu_batched_vae.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04i_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r04i_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/r04i_tests.log | head
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 --extras 0 --roofline-batch 0 > gpurun_out/r04i_bench.log 2>&1 || { tail -3 gpurun_out/r04i_bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r04i_bench.log').read().strip().splitlines()[-1]);print('fp32 step', round(d['ms_per_step'],3), 'ms')"
rm -rf gpurun_out/tr8192
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr8192 -o run -- python3 bench.py --steps 6 --warmup 2 --cpu-baseline 0 --extras 0 --roofline-batch 0 --batch 8192 > gpurun_out/tr8192.log 2>&1 || { tail -3 gpurun_out/tr8192.log; exit 1; }
f=$(ls gpurun_out/tr8192/*kernel_trace.csv gpurun_out/tr8192/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/step_timeline.py "$f" > gpurun_out/step8192_timeline.txt && python3 scripts/prof_step.py "$f" > gpurun_out/step8192.txt && tail -36 gpurun_out/step8192.txt
