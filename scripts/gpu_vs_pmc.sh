#!/bin/bash
# SQ counters of the fused bf16 step kernel (scripts/prof_one.py fused_bf16 65536 50),
# one rocprofv3 --pmc pass, under its own time limit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/vspmc
rm -rf $O; mkdir -p $O
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS --output-format csv -d $O/p1 -o run -- python3 scripts/prof_one.py fused_bf16 ${B:-65536} ${C:-50} > $O/p1.log 2>&1 || { echo "pass failed"; tail -3 $O/p1.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob("gpurun_out/vspmc/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "stn_vae_step_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:28s} {sum(v[-5:]) / len(v[-5:]):.4g}  (n={len(v)})")
PY
