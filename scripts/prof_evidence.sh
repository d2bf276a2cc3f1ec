#!/bin/bash
# Round profile (ROUND=r06 names the output directory and the evidence files): rocprofv3 --kernel-trace --stats of the default bench
# command, then per workload (scripts/prof_one.py) a kernel trace and separate
# FETCH_SIZE / WRITE_SIZE passes, each under its own time limit; stops at the
# first failure.  scripts/pmc_tables.py turns the passes into tables and the
# bench's pmc_summary.json entries.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${ROUND:-r06}
O=gpurun_out/${R}prof
rm -rf $O; mkdir -p $O
if [ "${SKIP_BENCH_TRACE:-0}" != 1 ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench -o run -- python3 bench.py > $O/bench.log 2>&1 || { echo "bench trace failed"; tail -5 $O/bench.log; exit 1; }
echo "bench trace ok"
fi
for W in "fused_bf16 65536 50" "fused_bf16 65536 64" "step_fp32 8192" "step_bf16 8192"; do
  N=$(echo $W | tr ' ' '_')
  timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $O/t_$N -o run -- python3 scripts/prof_one.py $W > $O/t_$N.log 2>&1 || { echo "trace $N failed"; tail -5 $O/t_$N.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_$N -o run -- python3 scripts/prof_one.py $W > $O/f_$N.log 2>&1 || { echo "fetch $N failed"; tail -5 $O/f_$N.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$N -o run -- python3 scripts/prof_one.py $W > $O/w_$N.log 2>&1 || { echo "write $N failed"; tail -5 $O/w_$N.log; exit 1; }
  echo "$N ok: $(tail -1 $O/t_$N.log)"
done
python3 scripts/pmc_tables.py $O $O/pmc_$R.json $R > $O/pmc_${R}_summary.txt && echo "summary ok"
