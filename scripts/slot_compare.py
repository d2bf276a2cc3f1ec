"""Per-kernel mean duration in each model's steps of a scripts/slot_trace.py
kernel trace (steps delimited by clip_adam; 15 per model), side by side."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "clip_adam" in r["Kernel_Name"]]
per = int(sys.argv[2]) if len(sys.argv) > 2 else 15
segs = []
for k in range(len(ends) // per):
    a = ends[k * per + 4] + 1  # after the warmup steps
    b = ends[k * per + per - 1] + 1
    d = collections.defaultdict(float)
    for r in rows[a:b]:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        n = n[:n.find("(")] if "(" in n else n
        d[n[:70]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 / (per - 5)
    span = (int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3 / (per - 5)
    segs.append((d, span))
print("span/step " + " ".join(f"{s:9.1f}" for _, s in segs))
keys = sorted(segs[0][0], key=lambda k: -segs[0][0][k])
for k in keys[:40]:
    print(" ".join(f"{d.get(k, 0):9.1f}" for d, _ in segs), " ", k)
