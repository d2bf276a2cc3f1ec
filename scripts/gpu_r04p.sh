#!/bin/bash
# full GPU suite, then every bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04p_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r04p_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/r04p_tests.log | head
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python3 bench.py > gpurun_out/r04p_bench.log 2>&1 || { tail -5 gpurun_out/r04p_bench.log; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/r04p_bench.log').read().strip().splitlines()[-1])
print('fp32', round(d['ms_per_step'],3), 'roof', d['roofline']['kernel'], round(d['roofline']['frac'],3))
for k,v in d.items():
    if isinstance(v,dict) and 'ms_per_step' in v: print(k, round(v['ms_per_step'],3))
    elif isinstance(v,dict) and 'frac' in v: print(k, round(v.get('avg_launch_us',v.get('avg_chain_us',0)),1), 'us frac', round(v['frac'],3))
PY
