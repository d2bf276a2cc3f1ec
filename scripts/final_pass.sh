#!/bin/bash
# Round-end GPU pass: the whole GPU suite, the default bench command under
# rocprofv3 --kernel-trace --stats (evidence for profiles/<round>_bench*), then the
# default bench line on its own.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
B64=0 bash scripts/gpu_quick.sh || exit 1
R=${ROUND:-r06}
O=gpurun_out/${R}prof
rm -rf $O/bench; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench -o run -- python3 bench.py > $O/bench.log 2>&1 || { echo "bench trace failed"; tail -5 $O/bench.log; exit 1; }
echo "bench trace ok"
TAG=${TAG:-${R}final} bash scripts/gpu_bench.sh > /dev/null || exit 1
python3 scripts/bench_summary.py gpurun_out/${TAG:-${R}final}_bench.log
