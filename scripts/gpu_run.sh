#!/bin/bash
# GPU-box runner: each step under its own timeout; stop on anything other than
# success (0) or an ordinary test failure (1) — faults/aborts/timeouts end the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1; shift
  local secs=$1; shift
  local t0=$(date +%s)
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc ($(( $(date +%s) - t0 ))s)"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
nc=0
for step in "$@"; do
  case "$step" in
    pytest) run pytest 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    pytestv) run pytest 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 400 python bench.py --steps 10 --warmup 3 --cpu-seconds 10 ;;
    benchq) run bench 300 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 ;;
    prof) run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 2 --cpu-baseline 0 ;;
    pmc) rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
         run pmcf 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --roofline-launches 3
         run pmcw 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --roofline-launches 3 ;;
    *) nc=$((nc + 1)); run custom$nc 600 bash -c "$step" ;;
  esac
done
