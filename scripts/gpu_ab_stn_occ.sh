#!/bin/bash
# STN backward at 4 waves / SIMD (11 VGPRs spilled) vs 3 (no spill): stand-alone and in the fp32 step.
# The A/B library is built beforehand, in mog-asr_amd/: stn.hip with __launch_bounds__(256, 3) on
# stn_bwd_kernel compiled to an object and linked with the other build/*.o into build_ab/libmog_air.so
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in 4 3 4 3; do
  L=""; [ $v = 3 ] && L=mog-asr_amd/build_ab/libmog_air.so
  MOG_AIR_LIB=$L timeout -k 10 120 python3 scripts/bench_stn.py 24576 > gpurun_out/stnocc_$v.log 2>&1 || { tail -3 gpurun_out/stnocc_$v.log; exit 1; }
  echo "occ $v: $(grep 'sep=True' gpurun_out/stnocc_$v.log)"
  MOG_AIR_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 --extras 0 --roofline-batch 0 > gpurun_out/stnocc_b$v.log 2>&1 || { tail -3 gpurun_out/stnocc_b$v.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/stnocc_b$v.log').read().strip().splitlines()[-1]);print('occ $v: fp32 step', round(d['ms_per_step'],3), 'ms')"
done
