#!/bin/bash
# the default bench (all lines) after the round-4 GEMM fixes, and the NT check
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 120 python3 scripts/x3nt_bench.py > gpurun_out/x3nt_r04n.log 2>&1 || { tail -5 gpurun_out/x3nt_r04n.log; exit 1; }
grep NT gpurun_out/x3nt_r04n.log
timeout -k 10 600 python3 bench.py > gpurun_out/r04n_bench.log 2>&1 || { tail -5 gpurun_out/r04n_bench.log; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/r04n_bench.log').read().strip().splitlines()[-1])
print('fp32', round(d['ms_per_step'],3), 'roof', d['roofline']['kernel'], round(d['roofline']['frac'],3))
for k,v in d.items():
    if isinstance(v,dict) and 'ms_per_step' in v: print(k, round(v['ms_per_step'],3))
    elif isinstance(v,dict) and 'frac' in v: print(k, round(v.get('avg_launch_us',v.get('avg_chain_us',0)),1), 'us frac', round(v['frac'],3))
print('cpu', d['cpu_baseline']['value'])
PY
