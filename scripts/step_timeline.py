"""Timeline of the last complete train step of a rocprofv3 kernel trace:
start / end (us from the step start), stream, grid, kernel."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "clip_adam" in r["Kernel_Name"]]
a, b = idx[-2] + 1, idx[-1] + 1
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:b]:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    n = n[:n.find("(")] if "(" in n else n
    g = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
    print(f"{s:8.1f} {e:8.1f} {e - s:7.1f}  q{r['Queue_Id']} s{r['Stream_Id']} g{g:<6} {n[:90]}")
