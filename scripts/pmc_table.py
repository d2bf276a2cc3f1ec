"""Sum rocprofv3 --pmc counters per kernel symbol over the passes in a
directory: python scripts/pmc_table.py <dir> [symbol-substring]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
agg, disp = {}, {}
for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(fn)):
        k = r["Kernel_Name"]
        if sub not in k:
            continue
        k = k.split("(")[0][-60:]
        agg.setdefault(k, {}).setdefault(r["Counter_Name"], 0.0)
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp.setdefault(k, set()).add(r["Dispatch_Id"])
for k, c in agg.items():
    n = len(disp[k])
    print(f"== {k}  dispatches={n}")
    for name in sorted(c):
        print(f"  {name:28s} {c[name] / n:16.1f} per dispatch")
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        for name in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if name in c:
                print(f"  {name} / WAVE_CYCLES = {c[name] / wc:.3f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "SQ_BUSY_CYCLES" in c:
        print(f"  MFMA_BUSY / BUSY_CYCLES = {c['SQ_VALU_MFMA_BUSY_CYCLES'] / c['SQ_BUSY_CYCLES']:.3f}")
