"""Average every counter of the dispatches of kernels matching a substring
across one or more rocprofv3 --pmc output directories.
usage: python scripts/pmc_kernel_table.py <substring> <dir> [<dir> ...]"""
import csv
import glob
import sys
from collections import defaultdict

sub = sys.argv[1]
vals = defaultdict(list)
dur = []
for d in sys.argv[2:]:
    for fn in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        per = defaultdict(dict)
        for r in csv.DictReader(open(fn)):
            if sub not in r["Kernel_Name"]:
                continue
            per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
            per[r["Dispatch_Id"]]["_dur"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            per[r["Dispatch_Id"]]["_grid"] = r["Grid_Size"]
        for e in per.values():
            for k, v in e.items():
                if k != "_grid":
                    vals[k].append(v)
for k in sorted(vals):
    v = vals[k]
    print(f"{k:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
